// k_tower.hip -- fp32 MFMA tower layer (BigDL Linear + ReLU chain) for gfx950.
//
// Restates model/encoder/HigherOrderEncoder.scala:34-59 (Linear(in->out, W: out x in,
// y = b + x W^T) + ReLU per fcDim, then Linear(->1)) and the output heads of
// DeepFM.scala:130-134 / XDeepFM / DCN / PNN (CAddTable + Sigmoid), on v_mfma_f32_16x16x4_f32
// (exact f32 FMA chain, 64 FLOP/clk/SIMD = the fp32 peak of the chip).
//
// Block = WM waves stacked on M, each wave owns 16 rows x all NT*16 columns of the block
// (NT accumulator tiles, 4*NT VGPRs).  With WM a multiple of 4 every SIMD carries the same
// number of waves, so the one barrier per K stage never waits on an overloaded SIMD.
// K is consumed in 16-wide chunks; inside a chunk lane group g = lane>>4 owns k = 4g..4g+3,
// so one ds_read_b128 per fragment feeds the 4 k-steps of the chunk.  LDS tiles are
// [rows][16] fp32 with a slot XOR-swizzle that keeps the 16-row fragment reads conflict-free
// for all four ds_read_b128 lane groups.  A stage holds BKC chunks; the next stage's global
// loads are issued before the MFMAs of the current one and written to LDS after them
// (register staging, one barrier per stage).
// The first layer may gather its A operand straight from the embedding table (ids staged in
// LDS): the gathered x = Reshape(B, F*k) of the embeddings is never materialised.
#include "rmx_internal.hpp"

namespace rmx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// physical 16-B slot of logical slot g in row `row` of a [rows][16] fp32 LDS tile
__device__ __forceinline__ int swz_slot(int row, int g) { return g ^ ((4 - ((row >> 2) & 3)) & 3); }

enum AMode : int { kDenseA = 0, kGatherK16 = 1, kGatherAny = 2 };

template <int NT, int WM, int BKC, int AMODE, int EPI>
__global__ __launch_bounds__(WM * 64) void tower_kernel(int M, int K, int Kpad, const float* __restrict__ A,
                                                         int lda, AGatherArgs ga, const float* __restrict__ Wp,
                                                         int Npad, const float* __restrict__ bias,
                                                         float* __restrict__ C, int ldc, OutArgs oa) {
  constexpr int BM = WM * 16, BN = NT * 16, NTHR = WM * 64;
  constexpr int AROWS = BM * BKC, ROWS = (BM + BN) * BKC;  // 64-B rows per stage
  constexpr int ITEMS = ROWS * 4;                            // float4 items per stage
  constexpr int PER = (ITEMS + NTHR - 1) / NTHR;
  constexpr int STAGE = ROWS * 16;                           // floats per stage

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lds0 = smem;
  float* lds1 = smem + STAGE;
  int* sids = reinterpret_cast<int*>(smem + 2 * STAGE);  // [BM][F] (gather modes)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = Kpad / 16;
  const int nstages = (nchunks + BKC - 1) / BKC;

  if constexpr (AMODE != kDenseA) {
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

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 stage[PER];
  // item i of a stage: row = i >> 2 (A rows first: [BKC][BM], then B rows [BKC][BN]), slot g = i & 3
  auto gload = [&](int st) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * NTHR;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int row = i >> 2, g = i & 3;
      if (row < AROWS) {
        const int cc = row / BM, r = row - cc * BM;
        const int c = st * BKC + cc;
        const int m = m0 + r;
        const int kk = c * 16 + g * 4;
        if (m < M && kk < K) {
          if constexpr (AMODE == kGatherK16) {
            const int id = sids[r * ga.F + c];
            v = *reinterpret_cast<const float4*>(ga.table + (int64_t)id * 16 + g * 4);
          } else if constexpr (AMODE == kGatherAny) {
            const int f = kk / ga.k, j = kk - f * ga.k;
            const int id = sids[r * ga.F + f];
            v = *reinterpret_cast<const float4*>(ga.table + (int64_t)id * ga.k + j);
          } else {
            v = *reinterpret_cast<const float4*>(A + (int64_t)m * lda + kk);
          }
        }
      } else if (row < ROWS) {
        const int rb = row - AROWS;
        const int cc = rb / BN, n = rb - cc * BN;
        const int c = st * BKC + cc;
        if (c < nchunks) v = *reinterpret_cast<const float4*>(Wp + ((int64_t)c * Npad + n0 + n) * 16 + g * 4);
      }
      stage[p] = v;
    }
  };
  auto sstore = [&](float* buf) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * NTHR;
      const int row = i >> 2, g = i & 3;
      if (row < ROWS) {
        const int lrow = row < AROWS ? (row % BM) : ((row - AROWS) % BN);
        *reinterpret_cast<float4*>(buf + row * 16 + swz_slot(lrow, g) * 4) = stage[p];
      }
    }
  };

  gload(0);
  sstore(lds0);
  __syncthreads();

  const int g = lane >> 4, r16 = lane & 15;
  const int arow = wid * 16 + r16;
  for (int st = 0; st < nstages; ++st) {
    const float* cur = (st & 1) ? lds1 : lds0;
    float* nxt = (st & 1) ? lds0 : lds1;
    if (st + 1 < nstages) gload(st + 1);
#pragma unroll
    for (int cc = 0; cc < BKC; ++cc) {
      const float* At = cur + cc * BM * 16;
      const float* Bt = cur + AROWS * 16 + cc * BN * 16;
      const float4 a = *reinterpret_cast<const float4*>(At + arow * 16 + swz_slot(arow, g) * 4);
#pragma unroll
      for (int j = 0; j < NT; j += 2) {
        const int row0 = j * 16 + r16;
        const float4 b0 = *reinterpret_cast<const float4*>(Bt + row0 * 16 + swz_slot(row0, g) * 4);
        if (j + 1 < NT) {
          const int row1 = row0 + 16;
          const float4 b1 = *reinterpret_cast<const float4*>(Bt + row1 * 16 + swz_slot(row1, g) * 4);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc[j], 0, 0, 0);
          acc[j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b1.x, acc[j + 1], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc[j], 0, 0, 0);
          acc[j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1.y, acc[j + 1], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc[j], 0, 0, 0);
          acc[j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b1.z, acc[j + 1], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc[j], 0, 0, 0);
          acc[j + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b1.w, acc[j + 1], 0, 0, 0);
        } else {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc[j], 0, 0, 0);
        }
      }
    }
    if (st + 1 < nstages) sstore(nxt);
    __syncthreads();
  }

  // C/D layout of 16x16 MFMA: lane holds rows 4*(lane>>4) + r (r = 0..3), column lane & 15.
  const int mw = m0 + wid * 16 + g * 4;
  if constexpr (EPI == static_cast<int>(Epi::kReluStore)) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + j * 16 + r16;
      const float bn = bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][r] + bn;
        v = v > 0.f ? v : 0.f;
        if (mw + r < M) C[(int64_t)(mw + r) * ldc + n] = v;
      }
    }
  } else {
    // Output head: logit = sum_n ReLU(acc + b)[n] * wo[n]; this block spans all of Npad.
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = j * 16 + r16;
      const float bn = bias[n], wo = oa.wo[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[j][r] + bn;
        v = v > 0.f ? v : 0.f;
        part[r] += v * wo;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = part[r];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      part[r] = v;
    }
    if (r16 < 4) {
      // lane r16 = r finalises row mw + r (rows of the lane group g)
      const int r = r16;
      const int m = mw + r;
      float y = r == 0 ? part[0] : (r == 1 ? part[1] : (r == 2 ? part[2] : part[3]));
      if (m < M) {
        if (oa.has_bo) y = y + oa.bo;
        if (oa.rowsum) {
          float rs = 0.f;
          for (int j = 0; j < oa.rowsum_k; ++j) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + j];
          y = rs + y;
        }
        if (oa.pre2) y = oa.pre2[m] + y;
        float t = oa.pre ? oa.pre[m] + y : y;
        t = t + oa.beta;
        oa.out[m] = 1.0f / (1.0f + expf(-t));
      }
    }
  }
}

// Output head for a last hidden layer too wide for one block: logit from the stored ReLU
// activations h[m][0..N) (one wave per row).
__global__ __launch_bounds__(256) void tower_head_kernel(int M, int N, const float* __restrict__ h, int ldh,
                                                         OutArgs oa) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float p = 0.f;
  for (int n = lane; n < N; n += 64) p += h[(int64_t)m * ldh + n] * oa.wo[n];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
  if (lane != 0) return;
  float y = p;
  if (oa.has_bo) y = y + oa.bo;
  if (oa.rowsum) {
    float rs = 0.f;
    for (int j = 0; j < oa.rowsum_k; ++j) rs += oa.rowsum[(int64_t)m * oa.rowsum_k + j];
    y = rs + y;
  }
  if (oa.pre2) y = oa.pre2[m] + y;
  float t = oa.pre ? oa.pre[m] + y : y;
  t = t + oa.beta;
  oa.out[m] = 1.0f / (1.0f + expf(-t));
}

// -------------------------------------------------------------- dispatch ----
namespace {

// column tiles per block that have kernels (a layer's Npad is a multiple of one of them)
constexpr int kNTs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 13, 16, 20, 25, 26};

template <int NT, int WM, int BKC, int AMODE, int EPI>
int launch_cfg(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda, const AGatherArgs* ga,
               float* C, int ldc, const OutArgs* oa) {
  constexpr int BM = WM * 16, BN = NT * 16;
  size_t lds = sizeof(float) * 2 * (BM + BN) * BKC * 16;
  AGatherArgs g{};
  if (AMODE != kDenseA) {
    g = *ga;
    lds += sizeof(int) * BM * g.F;
  }
  if (lds > 160 * 1024) {
    set_error("tower: LDS budget exceeded (" + std::to_string(lds) + " bytes)");
    return RMX_E_INVALID;
  }
  OutArgs o{};
  if (oa) o = *oa;
  dim3 grid((M + BM - 1) / BM, L.Npad / BN);
  auto kern = tower_kernel<NT, WM, BKC, AMODE, EPI>;
  if (lds > 64 * 1024)
    RMX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, grid, dim3(WM * 64), lds, s, M, L.K, L.Kpad, A, lda, g, L.W, L.Npad, L.b, C, ldc, o);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <int NT>
int launch_nt(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda, const AGatherArgs* ga, float* C,
              int ldc, Epi epi, const OutArgs* oa) {
  // 8 waves (2 per SIMD) for large batches, 4 for small ones; two K chunks per stage when the
  // A rows come from a dense activation buffer, one when they are gathered (ids share the LDS).
  const bool big = M >= 8192;
  const int amode = !ga ? kDenseA : (ga->k == 16 ? kGatherK16 : kGatherAny);
#define RMX_TOWER_CASE(WM, BKC, AM)                                                                   \
  if (epi == Epi::kReluStore) return launch_cfg<NT, WM, BKC, AM, 0>(s, L, M, A, lda, ga, C, ldc, oa); \
  return launch_cfg<NT, WM, BKC, AM, 1>(s, L, M, A, lda, ga, C, ldc, oa);
  if (big) {
    if (amode == kDenseA) { RMX_TOWER_CASE(8, 2, kDenseA) }
    if (amode == kGatherK16) { RMX_TOWER_CASE(8, 1, kGatherK16) }
    RMX_TOWER_CASE(8, 1, kGatherAny)
  }
  if (amode == kDenseA) { RMX_TOWER_CASE(4, 2, kDenseA) }
  if (amode == kGatherK16) { RMX_TOWER_CASE(4, 1, kGatherK16) }
  RMX_TOWER_CASE(4, 1, kGatherAny)
#undef RMX_TOWER_CASE
}

}  // namespace

// Npad of a layer of width N: a multiple of one block width NT*16 (NT from kNTs), chosen to
// minimise padding (ties: the wider block).
int tower_npad_for(int N) {
  const int nt = (N + 15) / 16;
  int best = -1, best_pad = 1 << 30;
  for (int c : kNTs) {
    const int pad = (nt + c - 1) / c * c;
    if (pad < best_pad || (pad == best_pad && c > best)) {
      best_pad = pad;
      best = c;
    }
  }
  return best_pad * 16;
}

int tower_nt_for(int Npad) {
  const int nt = Npad / 16;
  int best = 1;
  for (int c : kNTs)
    if (nt % c == 0 && c > best) best = c;
  return best;
}

int launch_tower_layer(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
                       const AGatherArgs* ga, float* C, int ldc, Epi epi, const OutArgs* oa) {
  if (M <= 0) return RMX_OK;
  const int nt = tower_nt_for(L.Npad);
  if (epi == Epi::kOutput && nt * 16 != L.Npad) {
    // too wide for one block: store the ReLU activations, then a separate head pass
    int st = launch_tower_layer(s, L, M, A, lda, ga, C, ldc, Epi::kReluStore, nullptr);
    if (st != RMX_OK) return st;
    hipLaunchKernelGGL(tower_head_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, L.N, C, ldc, *oa);
    RMX_HIP(hipGetLastError());
    return RMX_OK;
  }
  switch (nt) {
#define RMX_NT(n) \
  case n: return launch_nt<n>(s, L, M, A, lda, ga, C, ldc, epi, oa);
    RMX_NT(1) RMX_NT(2) RMX_NT(3) RMX_NT(4) RMX_NT(5) RMX_NT(6) RMX_NT(7)
    RMX_NT(8) RMX_NT(10) RMX_NT(13) RMX_NT(16) RMX_NT(20) RMX_NT(25) RMX_NT(26)
#undef RMX_NT
    default: set_error("bad tower width"); return RMX_E_INVALID;
  }
}

}  // namespace rmx
