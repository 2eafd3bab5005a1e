// k_cin.hip -- xDeepFM Compressed Interaction Network layer on fp32 MFMA (gfx950).
//
// Reference: model/xdeepfm/CINEncoder.scala:36-58, 105-176 (+ SURVEY.md Appendix A for L > 1):
//   x0[b,j,f] = e[b,f,j]                                  (shapeModule, :105-110)
//   z[f*Hp + h] = x0[b,j,f] * u_{l-1}[b,j,h]                (MM(transB = true), :152)
//   u_l[b,j,:] = ReLU(c_l + C_l z)                          (Linear + ReLU, :154-155)
//   pooled pi_l[b,h] = sum_j u_l[b,j,h]; y = W_out [pi_1 | ... | pi_L | d]   (:159-176)
//
// One launch per layer is a GEMM with M = B*k rows (b, j), K = F * Hp, N = H whose A operand is
// generated on the fly: the (F x Hp) outer product of a row is never materialised (the
// reference writes it: B*k x F*Hp floats, 2 GB per layer at B = 4096).  K is walked as
// h-chunks of 16 (outer) x fields f (inner): the row's u[h-chunk] stays in registers for all F
// fields, x0[row][f] comes from LDS, a = x0 * u is one VALU multiply per 4 MFMAs per tile.
// C_l is streamed through a double-buffered LDS stage in [chunk][N][16] packed order.
// Epilogue: ReLU, store u_l (next layer's input), and the output Linear folded in:
//   rowdot[b*k + j] (+)= sum_h u_l[b,j,h] * W_out[slice_l + h]
// which the tower's output head sums over j -- sum_j sum_h == sum_h (sum_j) = pi_l . W_out.
#include "rmx_models.hpp"

namespace rmx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int cin_swz(int row, int g) { return g ^ ((4 - ((row >> 2) & 3)) & 3); }

constexpr int kCinMT = 2, kCinWM = 4, kCinBM = kCinMT * kCinWM * 16, kCinThreads = kCinWM * 64;

template <int NT, bool FIRST>
__global__ __launch_bounds__(kCinThreads, 2) void cin_layer_kernel(
    int Mrows, int F, int k, int XS, int Hp_pad, const int32_t* __restrict__ ids, const float* __restrict__ table,
    const float* __restrict__ u_prev, const float* __restrict__ Wp, const float* __restrict__ cb,
    const float* __restrict__ wo, float* __restrict__ u_out, float* __restrict__ rowdot, int first_layer) {
  constexpr int NPAD = NT * 16;
  constexpr int ITEMS = NPAD * 4;
  constexpr int PER = (ITEMS + kCinThreads - 1) / kCinThreads;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* x0s = smem;                    // [BM][XS]
  float* w0 = smem + kCinBM * XS;       // [NPAD][16] x 2
  float* w1 = w0 + NPAD * 16;

  const int tid = threadIdx.x, lane = tid & 63, wm = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int m0 = blockIdx.x * kCinBM;

  // ---- x0 tile: x0s[r][f] = e[b, f, j] for row m0 + r = b*k + j; zero padded to XS columns.
  for (int i = tid; i < kCinBM * XS; i += kCinThreads) {
    const int j = i % k;
    const int rest = i / k;
    const int f = rest % XS;
    const int rb = rest / XS;  // sample slot within the block
    const int r = rb * k + j;
    if (r >= kCinBM) continue;
    const int m = m0 + r;
    float v = 0.f;
    if (f < F && m < Mrows) {
      const int b = m / k;
      const int id = ids ? ids[(int64_t)b * F + f] : b * F + f;
      v = table[(int64_t)id * k + j];
    }
    x0s[r * XS + f] = v;
  }

  f32x4 acc[kCinMT][NT];
#pragma unroll
  for (int i = 0; i < kCinMT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 stage[PER];
  auto gload = [&](int c) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * kCinThreads;
      if (i < ITEMS) stage[p] = *reinterpret_cast<const float4*>(Wp + (int64_t)c * NPAD * 16 + i * 4);
    }
  };
  auto sstore = [&](float* buf) {
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = tid + p * kCinThreads;
      if (i < ITEMS) {
        const int row = i >> 2, gg = i & 3;
        *reinterpret_cast<float4*>(buf + row * 16 + cin_swz(row, gg) * 4) = stage[p];
      }
    }
  };

  const int nchunks = (Hp_pad / 16) * F;
  gload(0);
  sstore(w0);
  __syncthreads();

  int rowl[kCinMT];
#pragma unroll
  for (int i = 0; i < kCinMT; ++i) rowl[i] = wm * kCinMT * 16 + i * 16 + r16;

  float4 uf[kCinMT];
  int hc = 0, f = 0;
  for (int c = 0; c < nchunks; ++c) {
    float* cur = (c & 1) ? w1 : w0;
    float* nxt = (c & 1) ? w0 : w1;
    if (c + 1 < nchunks) gload(c + 1);
    if (f == 0) {
#pragma unroll
      for (int i = 0; i < kCinMT; ++i) {
        if constexpr (FIRST) {
          uf[i] = *reinterpret_cast<const float4*>(x0s + rowl[i] * XS + hc * 16 + g * 4);
        } else {
          const int m = m0 + rowl[i];
          uf[i] = m < Mrows ? *reinterpret_cast<const float4*>(u_prev + (int64_t)m * Hp_pad + hc * 16 + g * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    float4 a[kCinMT];
#pragma unroll
    for (int i = 0; i < kCinMT; ++i) {
      const float xv = x0s[rowl[i] * XS + f];
      a[i] = make_float4(xv * uf[i].x, xv * uf[i].y, xv * uf[i].z, xv * uf[i].w);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = j * 16 + r16;
      const float4 b = *reinterpret_cast<const float4*>(cur + row * 16 + cin_swz(row, g) * 4);
#pragma unroll
      for (int i = 0; i < kCinMT; ++i) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b.x, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b.y, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b.z, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b.w, acc[i][j], 0, 0, 0);
      }
    }
    if (c + 1 < nchunks) sstore(nxt);
    __syncthreads();
    if (++f == F) {
      f = 0;
      ++hc;
    }
  }

  // ---- epilogue: C/D lane map rows 4*g + r, column r16.
  float part[kCinMT][4];
#pragma unroll
  for (int i = 0; i < kCinMT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = j * 16 + r16;
    const float bn = cb[n], wn = wo[n];
#pragma unroll
    for (int i = 0; i < kCinMT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] + bn;
        v = v > 0.f ? v : 0.f;
        part[i][r] += v * wn;
        const int m = m0 + wm * kCinMT * 16 + i * 16 + g * 4 + r;
        if (u_out && m < Mrows) u_out[(int64_t)m * NPAD + n] = v;
      }
  }
#pragma unroll
  for (int i = 0; i < kCinMT; ++i)
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
    for (int i = 0; i < kCinMT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * kCinMT * 16 + i * 16 + g * 4 + r;
        if (m < Mrows) rowdot[m] = first_layer ? part[i][r] : rowdot[m] + part[i][r];
      }
  }
}

// C_l (H x F*Hp row-major, column f*Hp + h) -> [Hp_pad/16][F][Npad][16]
__global__ void pack_cin_kernel(const float* __restrict__ C, int F, int Hp, int H, int Npad, int64_t tot,
                                float* __restrict__ Wp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int kk = (int)(i & 15);
  const int64_t rest = i >> 4;
  const int n = (int)(rest % Npad);
  const int64_t c = rest / Npad;
  const int f = (int)(c % F);
  const int hc = (int)(c / F);
  const int h = hc * 16 + kk;
  Wp[i] = (n < H && h < Hp) ? C[(int64_t)n * F * Hp + (int64_t)f * Hp + h] : 0.f;
}

int launch_pack_cin(hipStream_t s, const float* mats, int F, CinLayer& L) {
  const int64_t tot = (int64_t)L.Hp_pad * F * L.Npad;
  hipLaunchKernelGGL(pack_cin_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats + L.w_off, F,
                     L.Hp, L.H, L.Npad, tot, L.W);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

namespace {
template <int NT>
int launch_nt(hipStream_t s, const CinLayer& L, bool first, bool last, int B, int F, int k, const int32_t* ids,
              const float* table, const float* u_prev, float* u_out, float* rowdot) {
  const int Mrows = B * k;
  const int XS = round_up(F, 16) + 4;  // 16-B aligned rows; XS/4 odd spreads the scalar reads
  const size_t lds = sizeof(float) * ((size_t)kCinBM * XS + 2 * NT * 16 * 16);
  dim3 grid((Mrows + kCinBM - 1) / kCinBM);
  if (first) {
    auto kern = cin_layer_kernel<NT, true>;
    if (lds > 64 * 1024)
      RMX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, grid, dim3(kCinThreads), lds, s, Mrows, F, k, XS, L.Hp_pad, ids, table, u_prev,
                       L.W, L.b, L.wo, last ? nullptr : u_out, rowdot, 1);
  } else {
    auto kern = cin_layer_kernel<NT, false>;
    if (lds > 64 * 1024)
      RMX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, grid, dim3(kCinThreads), lds, s, Mrows, F, k, XS, L.Hp_pad, ids, table, u_prev,
                       L.W, L.b, L.wo, last ? nullptr : u_out, rowdot, 0);
  }
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}
}  // namespace

int launch_cin_layer(hipStream_t s, const CinLayer& L, bool first, bool last, int B, int F, int k,
                     const int32_t* ids, const float* table, const float* u_prev, float* u_out, float* rowdot) {
  if (B <= 0) return RMX_OK;
  if (!first && !u_prev) {
    set_error("cin: missing previous layer maps");
    return RMX_E_INVALID;
  }
  if (first && L.Hp_pad > round_up(F, 16)) {
    set_error("cin: first layer Hp_pad mismatch");
    return RMX_E_INVALID;
  }
  switch (L.Npad / 16) {
#define CASE(n) \
  case n: return launch_nt<n>(s, L, first, last, B, F, k, ids, table, u_prev, u_out, rowdot);
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default:
      set_error("cin: layer width must be <= 256");
      return RMX_E_INVALID;
  }
}

}  // namespace rmx
