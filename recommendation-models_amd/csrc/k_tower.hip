// k_tower.hip -- fp32 MFMA tower layer (BigDL Linear + ReLU chain) for gfx950.
//
// Restates model/encoder/HigherOrderEncoder.scala:34-59 (Linear(in->out, W: out x in,
// y = b + x W^T) + ReLU per fcDim, then Linear(->1)) and the output heads of
// DeepFM.scala:130-134 / XDeepFM / DCN / PNN (CAddTable + Sigmoid), on v_mfma_f32_16x16x4_f32
// (exact f32 FMA chain, 64 FLOP/clk/SIMD = the fp32 peak of the chip).
//
// Block = WN waves side by side on N (each wave NT 16x16 tiles) x MT 16-row tiles on M.
// K is consumed in 16-wide chunks; inside a chunk lane group g = lane>>4 owns k = 4g..4g+3,
// so one ds_read_b128 per fragment feeds the 4 k-steps of the chunk.  The LDS tiles are
// [rows][16] fp32 with a slot XOR-swizzle that makes the 16-row fragment reads
// conflict-free for all four ds_read_b128 lane groups.
// The first layer may gather its A operand straight from the embedding table (ids staged in
// LDS): the gathered x = Reshape(B, F*k) of the embeddings is never materialised.
#include "rmx_internal.hpp"

namespace rmx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// physical 16-B slot of logical slot g in row `row` of a [rows][16] fp32 LDS tile
__device__ __forceinline__ int swz_slot(int row, int g) { return g ^ ((4 - ((row >> 2) & 3)) & 3); }

template <int MT, int NT, int WM, int WN, bool GATHER, bool K16, int EPI>
__global__ __launch_bounds__(WM* WN * 64) void tower_layer_kernel(
    int M, int K, int Kpad, const float* __restrict__ A, int lda, AGatherArgs ga,
    const float* __restrict__ Wp, int Npad, const float* __restrict__ bias, float* __restrict__ C,
    int ldc, OutArgs oa) {
  constexpr int BM = WM * MT * 16, BN = WN * NT * 16, NTHR = WM * WN * 64;
  constexpr int AITEMS = BM * 4, ITEMS = (BM + BN) * 4;
  constexpr int PER = (ITEMS + NTHR - 1) / NTHR;
  constexpr int TILE = (BM + BN) * 16;  // floats per LDS stage

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lds0 = smem;
  float* lds1 = smem + TILE;
  int* sids = reinterpret_cast<int*>(smem + 2 * TILE);  // [BM][F] (GATHER only)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = Kpad / 16;

  if constexpr (GATHER) {
    const int F = ga.F;
    for (int i = tid; i < BM * F; i += NTHR) {
      const int r = i / F, f = i - r * F;
      const int m = m0 + r;
      int id = 0;
      if (m < M) id = ga.ids ? ga.ids[(int64_t)m * F + f] : m * F + f;
      sids[i] = id;
    }
    __syncthreads();
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 stage[PER];

  auto gload = [&](int c) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * NTHR;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < AITEMS) {
        const int row = i >> 2, g = i & 3;
        const int m = m0 + row;
        const int kk = c * 16 + g * 4;
        if (m < M && kk < K) {
          if constexpr (GATHER) {
            int f, j;
            if constexpr (K16) {
              f = c;
              j = g * 4;
            } else {
              f = kk / ga.k;
              j = kk - f * ga.k;
            }
            const int id = sids[row * ga.F + f];
            v = *reinterpret_cast<const float4*>(ga.table + (int64_t)id * ga.k + j);
          } else {
            v = *reinterpret_cast<const float4*>(A + (int64_t)m * lda + kk);
          }
        }
      } else if (i < ITEMS) {
        const int jb = i - AITEMS;
        const int row = jb >> 2, g = jb & 3;
        v = *reinterpret_cast<const float4*>(Wp + ((int64_t)c * Npad + n0 + row) * 16 + g * 4);
      }
      stage[p] = v;
    }
  };
  auto sstore = [&](float* buf) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * NTHR;
      if (i < ITEMS) {
        int row, g, base;
        if (i < AITEMS) {
          row = i >> 2;
          g = i & 3;
          base = 0;
        } else {
          row = (i - AITEMS) >> 2;
          g = (i - AITEMS) & 3;
          base = BM * 16;
        }
        *reinterpret_cast<float4*>(buf + base + row * 16 + swz_slot(row, g) * 4) = stage[p];
      }
    }
  };

  gload(0);
  sstore(lds0);
  __syncthreads();

  const int g = lane >> 4, r16 = lane & 15;
  for (int c = 0; c < nchunks; ++c) {
    float* cur = (c & 1) ? lds1 : lds0;
    float* nxt = (c & 1) ? lds0 : lds1;
    if (c + 1 < nchunks) gload(c + 1);
    float4 a[MT], b[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int row = wm * MT * 16 + i * 16 + r16;
      a[i] = *reinterpret_cast<const float4*>(cur + row * 16 + swz_slot(row, g) * 4);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = wn * NT * 16 + j * 16 + r16;
      b[j] = *reinterpret_cast<const float4*>(cur + BM * 16 + row * 16 + swz_slot(row, g) * 4);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
      }
    if (c + 1 < nchunks) sstore(nxt);
    __syncthreads();
  }

  // C/D layout of 16x16 MFMA: lane holds rows 4*(lane>>4) + r (r = 0..3), column lane & 15.
  if constexpr (EPI == static_cast<int>(Epi::kReluStore)) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + wn * NT * 16 + j * 16 + r16;
        const float bn = bias[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * MT * 16 + i * 16 + g * 4 + r;
          float v = acc[i][j][r] + bn;
          v = v > 0.f ? v : 0.f;
          if (m < M) C[(int64_t)m * ldc + n] = v;
        }
      }
  } else {
    // Output head: logit = sum_n ReLU(acc + b)[n] * wo[n]; this block spans all of Npad.
    float* red = smem;  // reuse stage buffers: [WN][BM]
    float part[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[i][r] = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + wn * NT * 16 + j * 16 + r16;
      const float bn = bias[n], wo = oa.wo[n];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bn;
          v = v > 0.f ? v : 0.f;
          part[i][r] += v * wo;
        }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = part[i][r];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        part[i][r] = v;
      }
    if (r16 == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wn * BM + wm * MT * 16 + i * 16 + g * 4 + r] = part[i][r];
    }
    __syncthreads();
    for (int rr = tid; rr < BM; rr += NTHR) {
      const int m = m0 + rr;
      if (m >= M) continue;
      float y = 0.f;
#pragma unroll
      for (int w = 0; w < WN; ++w) y += red[w * BM + rr];
      if (oa.has_bo) y = y + oa.bo;
      if (oa.rowsum) {
        float r = 0.f;
        for (int j = 0; j < oa.rowsum_k; ++j) r += oa.rowsum[(int64_t)m * oa.rowsum_k + j];
        y = r + y;
      }
      if (oa.pre2) y = oa.pre2[m] + y;
      float t = oa.pre ? oa.pre[m] + y : y;
      t = t + oa.beta;
      oa.out[m] = 1.0f / (1.0f + expf(-t));
    }
  }
}

// -------------------------------------------------------------- dispatch ----
namespace {

constexpr int kMT = 4, kNT = 5, kWM = 1;

template <int WN, bool GATHER, bool K16, int EPI>
int launch_cfg(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
               const AGatherArgs* ga, float* C, int ldc, const OutArgs* oa) {
  constexpr int BM = kWM * kMT * 16, BN = WN * kNT * 16, NTHR = kWM * WN * 64;
  constexpr int TILE = (BM + BN) * 16;
  size_t lds = sizeof(float) * 2 * TILE;
  AGatherArgs g{};
  if (GATHER) {
    g = *ga;
    lds += sizeof(int) * BM * g.F;
  }
  if (EPI == static_cast<int>(Epi::kOutput)) {
    const size_t red = sizeof(float) * WN * BM;
    if (red > lds) lds = red;
  }
  OutArgs o{};
  if (oa) o = *oa;
  dim3 grid((M + BM - 1) / BM, L.Npad / BN);
  auto kern = tower_layer_kernel<kMT, kNT, kWM, WN, GATHER, K16, EPI>;
  if (lds > 64 * 1024) RMX_HIP(hipFuncSetAttribute((const void*)kern,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)lds));
  hipLaunchKernelGGL(kern, grid, dim3(NTHR), lds, s, M, L.K, L.Kpad, A, lda, g, L.W, L.Npad, L.b,
                     C, ldc, o);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <int WN>
int launch_wn(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
              const AGatherArgs* ga, float* C, int ldc, Epi epi, const OutArgs* oa) {
  const bool k16 = ga && ga->k == 16;
  if (epi == Epi::kReluStore) {
    if (!ga) return launch_cfg<WN, false, false, 0>(s, L, M, A, lda, ga, C, ldc, oa);
    if (k16) return launch_cfg<WN, true, true, 0>(s, L, M, A, lda, ga, C, ldc, oa);
    return launch_cfg<WN, true, false, 0>(s, L, M, A, lda, ga, C, ldc, oa);
  }
  if (!ga) return launch_cfg<WN, false, false, 1>(s, L, M, A, lda, ga, C, ldc, oa);
  if (k16) return launch_cfg<WN, true, true, 1>(s, L, M, A, lda, ga, C, ldc, oa);
  return launch_cfg<WN, true, false, 1>(s, L, M, A, lda, ga, C, ldc, oa);
}

}  // namespace

// Npad of every packed layer is a multiple of 80 (= NT * 16); the block spans
// WN = min(Npad / 80, 8) waves on N, more N-blocks beyond that (ReLU-store only).
int tower_wn_for(int Npad) {
  int wn = Npad / (kNT * 16);
  while (wn > 8 || (Npad / (kNT * 16)) % wn) --wn;
  return wn;
}

int launch_tower_layer(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
                       const AGatherArgs* ga, float* C, int ldc, Epi epi, const OutArgs* oa) {
  if (M <= 0) return RMX_OK;
  const int wn = tower_wn_for(L.Npad);
  if (epi == Epi::kOutput && wn * kNT * 16 != L.Npad) {
    set_error("output head needs the whole layer width in one block (Npad <= 640)");
    return RMX_E_INVALID;
  }
  switch (wn) {
    case 1: return launch_wn<1>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 2: return launch_wn<2>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 3: return launch_wn<3>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 4: return launch_wn<4>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 5: return launch_wn<5>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 6: return launch_wn<6>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 7: return launch_wn<7>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    case 8: return launch_wn<8>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    default: set_error("bad tower width"); return RMX_E_INVALID;
  }
}

}  // namespace rmx
