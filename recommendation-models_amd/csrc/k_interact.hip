// k_interact.hip -- DCN cross network and PNN inner-product encoder (gfx950).
//
// DCN  model/dcn/CrossEncoder.scala:40-55, 107-152:
//   x_{l+1} = ((x0 * (w_l . x_l)) + x_l) + beta_l   (Linear(D->1, no bias), MM, CAddTable, CAdd(1))
//   the x_L slice of the output Linear (:176-185) is folded in: pre2[b] = x_L . W_out[0:D].
//   One wave per sample; x0 / x_l live in registers (D <= 1024 -> <= 16 per lane).
// PNN  model/pnn/ProductEncoder.scala:84-120, bnn/Gather.scala:19-47, bnn/DotProduct2.scala:16-26:
//   ip[b,p] = sum_t e[b,i_p,t] * e[b,j_p,t] over pairs (i < j) in lexicographic order;
//   writes the row [x | ip] (zero padded) that feeds ONE GEMM for Wz x + Wp ip (K = D + P).
#include <algorithm>

#include "rmx_models.hpp"

namespace rmx {

constexpr int kCrossNPL = 16;  // D <= 64 * 16

__device__ __forceinline__ float wave_sum(float v) {
  v += __shfl_xor(v, 32);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

template <class T>
__global__ __launch_bounds__(256) void cross_kernel(int B, int F, int k, int L, const int32_t* __restrict__ ids,
                                                    const T* __restrict__ table,
                                                    const float* __restrict__ cross_w,
                                                    const float* __restrict__ cross_b,
                                                    const float* __restrict__ wo_x, float* __restrict__ pre2) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int D = F * k;
  float x0[kCrossNPL], xl[kCrossNPL];
#pragma unroll
  for (int i = 0; i < kCrossNPL; ++i) {
    const int d = lane + 64 * i;
    float v = 0.f;
    if (d < D) {
      const int f = d / k, j = d - (d / k) * k;
      const int id = ids ? ids[(int64_t)b * F + f] : b * F + f;
      v = ld1(table + (int64_t)id * k + j);
    }
    x0[i] = v;
    xl[i] = v;
  }
  for (int l = 0; l < L; ++l) {
    const float* w = cross_w + (int64_t)l * D;
    float p = 0.f;
#pragma unroll
    for (int i = 0; i < kCrossNPL; ++i) {
      const int d = lane + 64 * i;
      if (d < D) p += xl[i] * w[d];
    }
    const float s = wave_sum(p);
    const float bl = cross_b[l];
#pragma unroll
    for (int i = 0; i < kCrossNPL; ++i) xl[i] = ((x0[i] * s) + xl[i]) + bl;
  }
  float p = 0.f;
#pragma unroll
  for (int i = 0; i < kCrossNPL; ++i) {
    const int d = lane + 64 * i;
    if (d < D) p += xl[i] * wo_x[d];
  }
  const float y = wave_sum(p);
  if (lane == 0) pre2[b] = y;
}

// k = 16: 16 lanes per sample (lane j holds column j of every field: x0[f], x_l[f] for f < F in
// registers), 4 samples per wave.  Every row load is one coalesced 64-B (32-B bf16) segment per
// 16 lanes; the per-layer dot is a 16-lane butterfly; the cross vectors are staged in LDS once
// per block.  FMAX bounds F at compile time (registers).
template <class T, int FMAX>
__global__ __launch_bounds__(256) void cross16_kernel(int B, int F, int L, const int32_t* __restrict__ ids,
                                                      const T* __restrict__ table,
                                                      const float* __restrict__ cross_w,
                                                      const float* __restrict__ cross_b,
                                                      const float* __restrict__ wo_x, float* __restrict__ pre2) {
  extern __shared__ __attribute__((aligned(16))) float wsh[];  // [L + 1][D]: w_1..w_L, W_out[0:D]
  const int D = F * 16;
  for (int i = threadIdx.x; i < (L + 1) * D; i += blockDim.x)
    wsh[i] = i < L * D ? cross_w[i] : wo_x[i - L * D];
  __syncthreads();
  const int j = threadIdx.x & 15;
  const int b = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (b >= B) return;  // no barrier follows
  float x0[FMAX], xl[FMAX];
#pragma unroll
  for (int f = 0; f < FMAX; ++f) {
    float v = 0.f;
    if (f < F) v = ld1(table + (int64_t)ids[(int64_t)b * F + f] * 16 + j);
    x0[f] = v;
    xl[f] = v;
  }
  auto dot16 = [&](const float* w) {
    float p = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f)
      if (f < F) p += xl[f] * w[f * 16 + j];
    p += __shfl_xor(p, 1);
    p += __shfl_xor(p, 2);
    p += __shfl_xor(p, 4);
    p += __shfl_xor(p, 8);
    return p;
  };
  for (int l = 0; l < L; ++l) {
    const float sdot = dot16(wsh + l * D);
    const float bl = cross_b[l];
#pragma unroll
    for (int f = 0; f < FMAX; ++f) xl[f] = ((x0[f] * sdot) + xl[f]) + bl;
  }
  const float y = dot16(wsh + L * D);
  if (j == 0) pre2[b] = y;
}

// Cross stack in closed form from the fused dot products (DCN layer 1 carries x0.w_l and x0.W_out[0:D]
// as raw extra GEMM columns): with x_l = a_l x0 + c_l 1, s_l = w_l.x_l = a_l u_l + c_l sum(w_l),
// a_{l+1} = a_l + s_l, c_{l+1} = c_l + beta_l, and x_L.W_out[0:D] = a_L v + c_L sum(W_out[0:D]).
// Exact algebra of CrossEncoder.scala:44-49; only the fp32 summation order differs.
__global__ void cross_finish_kernel(int B, int L, const float* __restrict__ xcol, CrossScalars cs,
                                    float* __restrict__ pre2) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* u = xcol + (int64_t)b * (L + 1);
  float a = 1.f, c = 0.f;
  for (int l = 0; l < L; ++l) {
    const float sl = a * u[l] + c * cs.wsum[l];
    a = a + sl;
    c = c + cs.beta[l];
  }
  pre2[b] = a * u[L] + c * cs.wo_sum;
}

int launch_cross_finish(hipStream_t s, int B, int L, const float* xcol, const CrossScalars& cs, float* pre2) {
  if (B <= 0) return RMX_OK;
  hipLaunchKernelGGL(cross_finish_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, L, xcol, cs, pre2);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

int launch_cross(hipStream_t s, int B, int F, int k, int L, const int32_t* ids, const void* table, int dt,
                 const float* cross_w, const float* cross_b, const float* wo_x, float* pre2) {
  if (B <= 0) return RMX_OK;
  if (k == 16 && F <= 64 && ids) {
    const size_t lds = sizeof(float) * (L + 1) * F * 16;
    if (lds <= 64 * 1024) {
      const dim3 grid((B + 15) / 16), blk(256);
#define RMX_CROSS(FM)                                                                                             \
  if (dt == kBF16)                                                                                                \
    hipLaunchKernelGGL((cross16_kernel<bf16_t, FM>), grid, blk, lds, s, B, F, L, ids, (const bf16_t*)table, cross_w, \
                       cross_b, wo_x, pre2);                                                                     \
  else                                                                                                            \
    hipLaunchKernelGGL((cross16_kernel<float, FM>), grid, blk, lds, s, B, F, L, ids, (const float*)table, cross_w,   \
                       cross_b, wo_x, pre2);
      if (F <= 16) { RMX_CROSS(16) } else if (F <= 40) { RMX_CROSS(40) } else { RMX_CROSS(64) }
#undef RMX_CROSS
      RMX_HIP(hipGetLastError());
      return RMX_OK;
    }
  }
  if (F * k > 64 * kCrossNPL) {
    set_error("cross: nFields * embeddingDim must be <= 1024");
    return RMX_E_INVALID;
  }
  if (dt == kBF16)
    hipLaunchKernelGGL(cross_kernel<bf16_t>, dim3((B + 3) / 4), dim3(256), 0, s, B, F, k, L, ids,
                       (const bf16_t*)table, cross_w, cross_b, wo_x, pre2);
  else
    hipLaunchKernelGGL(cross_kernel<float>, dim3((B + 3) / 4), dim3(256), 0, s, B, F, k, L, ids,
                       (const float*)table, cross_w, cross_b, wo_x, pre2);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// T: table elements; X: [x | ip] row elements (bf16 rows feed the bf16 GEMM: ip rounded once)
template <class T, class X>
__global__ __launch_bounds__(256) void product_kernel(int B, int F, int k, const int32_t* __restrict__ ids,
                                                      const T* __restrict__ table,
                                                      const int32_t* __restrict__ pairs, int P,
                                                      X* __restrict__ xbuf, int ldx) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float es[];
  const int D = F * k;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + w;
  float* e = es + w * (D + 1);
  if (b < B) {
    for (int d = lane; d < D; d += 64) {
      const int f = d / k, j = d - f * k;
      const int id = ids ? ids[(int64_t)b * F + f] : b * F + f;
      const float v = ld1(table + (int64_t)id * k + j);
      e[d] = v;
      st1(xbuf + (int64_t)b * ldx + d, v);
    }
  }
  __syncthreads();
  if (b >= B) return;
  for (int p = lane; p < P; p += 64) {
    const int i = pairs[2 * p], j = pairs[2 * p + 1];
    float acc = 0.f;
    for (int t = 0; t < k; ++t) acc += e[i * k + t] * e[j * k + t];
    st1(xbuf + (int64_t)b * ldx + D + p, acc);
  }
  for (int c = D + P + lane; c < ldx; c += 64) st1(xbuf + (int64_t)b * ldx + c, 0.f);
}

// k = 16: the pair products of a sample are its Gram matrix G = E E^T (F x F, K = 16) on
// v_mfma_f32_16x16x4_f32.  Lane (r16, g) gathers E[16t + r16][4g .. 4g+3] of every 16-row tile t
// straight from the table into registers; that one fragment is both the A operand (rows of tile I)
// and the B operand (E^T columns of tile J), so the NTILE(NTILE+1)/2 upper tiles cost 4 MFMAs each
// and no LDS.  Each lane writes its x fragment (16 B) and, for row i of its G tile, the pair slots
// p(i, j) = i(2F-i-1)/2 + j-i-1 of 16 consecutive j (one contiguous segment per 16 lanes).
// One wave per sample, grid-strided.
// 16-byte stores of the [x | ip] row: 8 bf16 or 4 fp32 per lane-store
template <class X>
struct Vec16;
template <>
struct Vec16<bf16_t> {
  static constexpr int N = 8;
};
template <>
struct Vec16<float> {
  static constexpr int N = 4;
};

template <class T, class X, int NTILE>
__global__ __launch_bounds__(256) void product16_kernel(int B, int F, const int32_t* __restrict__ ids,
                                                        const T* __restrict__ table, X* __restrict__ xbuf, int ldx) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  typedef X xvec4 __attribute__((ext_vector_type(4)));
  // the wave's [ip | zero pad] segment of the row, assembled in LDS and written with 16-B stores
  // (the pair slots of one G tile row are 2-B scattered writes otherwise)
  constexpr int kSeg = 64 * 63 / 2 + 32;
  __shared__ __attribute__((aligned(16))) X seg[4][kSeg];
  const int lane = threadIdx.x & 63, g = lane >> 4, r16 = lane & 15;
  X* sw = seg[threadIdx.x >> 6];
  const int D = F * 16;
  const int P = F * (F - 1) / 2;
  const int nw = gridDim.x * 4;
  for (int b = blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += nw) {
    X* xr = xbuf + (int64_t)b * ldx;
    f32x4 fr[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const int row = t * 16 + r16;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < F) {
        v = load4(table + (int64_t)ids[(int64_t)b * F + row] * 16 + g * 4);
        xvec4 xv;
        xv[0] = (X)v.x;
        xv[1] = (X)v.y;
        xv[2] = (X)v.z;
        xv[3] = (X)v.w;
        *reinterpret_cast<xvec4*>(xr + row * 16 + g * 4) = xv;
      }
      fr[t] = f32x4{v.x, v.y, v.z, v.w};
    }
    for (int c = P + lane; c < ldx - D; c += 64) sw[c] = (X)0.f;
#pragma unroll
    for (int I = 0; I < NTILE; ++I)
#pragma unroll
      for (int J = I; J < NTILE; ++J) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fr[I][s4], fr[J][s4], acc, 0, 0, 0);
        const int j = J * 16 + r16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = I * 16 + g * 4 + r;
          if (i < j && j < F) sw[i * (2 * F - i - 1) / 2 + (j - i - 1)] = (X)acc[r];
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS writes, before its lanes read them
    constexpr int VN = Vec16<X>::N;
    for (int c = lane * VN; c < ldx - D; c += 64 * VN)
      *reinterpret_cast<float4*>(xr + D + c) = *reinterpret_cast<const float4*>(sw + c);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next sample's writes
  }
}

int launch_product(hipStream_t s, int B, int F, int k, const int32_t* ids, const void* table, int dt,
                   const int32_t* pairs, int P, void* xbuf, int xdt, int ldx) {
  if (B <= 0) return RMX_OK;
  if (k == 16 && F <= 64 && ids && ldx - F * 16 <= 64 * 63 / 2 + 32) {
    const int nblk = std::min((B + 3) / 4, 256 * 16);
    const dim3 grid(nblk), blk(256);
#define RMX_PROD(NTL)                                                                                              \
  if (dt == kBF16 && xdt == kBF16)                                                                                 \
    hipLaunchKernelGGL((product16_kernel<bf16_t, bf16_t, NTL>), grid, blk, 0, s, B, F, ids, (const bf16_t*)table,  \
                       (bf16_t*)xbuf, ldx);                                                                        \
  else if (dt == kBF16)                                                                                            \
    hipLaunchKernelGGL((product16_kernel<bf16_t, float, NTL>), grid, blk, 0, s, B, F, ids, (const bf16_t*)table,   \
                       (float*)xbuf, ldx);                                                                         \
  else if (xdt == kBF16)                                                                                           \
    hipLaunchKernelGGL((product16_kernel<float, bf16_t, NTL>), grid, blk, 0, s, B, F, ids, (const float*)table,    \
                       (bf16_t*)xbuf, ldx);                                                                        \
  else                                                                                                             \
    hipLaunchKernelGGL((product16_kernel<float, float, NTL>), grid, blk, 0, s, B, F, ids, (const float*)table,     \
                       (float*)xbuf, ldx);
    const int nt = (F + 15) / 16;
    if (nt == 1) { RMX_PROD(1) } else if (nt == 2) { RMX_PROD(2) } else if (nt == 3) { RMX_PROD(3) } else { RMX_PROD(4) }
#undef RMX_PROD
    RMX_HIP(hipGetLastError());
    return RMX_OK;
  }
  const size_t lds = sizeof(float) * 4 * (F * k + 1);
  const dim3 grid((B + 3) / 4), blk(256);
  if (dt == kBF16 && xdt == kBF16)
    hipLaunchKernelGGL((product_kernel<bf16_t, bf16_t>), grid, blk, lds, s, B, F, k, ids, (const bf16_t*)table, pairs,
                       P, (bf16_t*)xbuf, ldx);
  else if (dt == kBF16)
    hipLaunchKernelGGL((product_kernel<bf16_t, float>), grid, blk, lds, s, B, F, k, ids, (const bf16_t*)table, pairs,
                       P, (float*)xbuf, ldx);
  else if (xdt == kBF16)
    hipLaunchKernelGGL((product_kernel<float, bf16_t>), grid, blk, lds, s, B, F, k, ids, (const float*)table, pairs,
                       P, (bf16_t*)xbuf, ldx);
  else
    hipLaunchKernelGGL((product_kernel<float, float>), grid, blk, lds, s, B, F, k, ids, (const float*)table, pairs, P,
                       (float*)xbuf, ldx);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <class T, class X>
__global__ void gather_x_kernel(int B, int F, int k, const int32_t* __restrict__ ids,
                                const T* __restrict__ table, X* __restrict__ xbuf, int ldx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * ldx) return;
  const int64_t b = i / ldx;
  const int d = (int)(i - b * ldx);
  float v = 0.f;
  if (d < F * k) {
    const int f = d / k, j = d - f * k;
    const int id = ids ? ids[b * F + f] : (int)(b * F + f);
    v = ld1(table + (int64_t)id * k + j);
  }
  st1(xbuf + i, v);
}

int launch_gather_x(hipStream_t s, int B, int F, int k, const int32_t* ids, const void* table, int dt, void* xbuf,
                    int xdt, int ldx) {
  const int64_t tot = (int64_t)B * ldx;
  if (tot <= 0) return RMX_OK;
  const dim3 grid((unsigned)((tot + 255) / 256)), blk(256);
  if (dt == kBF16 && xdt == kBF16)
    hipLaunchKernelGGL((gather_x_kernel<bf16_t, bf16_t>), grid, blk, 0, s, B, F, k, ids, (const bf16_t*)table,
                       (bf16_t*)xbuf, ldx);
  else if (dt == kBF16)
    hipLaunchKernelGGL((gather_x_kernel<bf16_t, float>), grid, blk, 0, s, B, F, k, ids, (const bf16_t*)table,
                       (float*)xbuf, ldx);
  else if (xdt == kBF16)
    hipLaunchKernelGGL((gather_x_kernel<float, bf16_t>), grid, blk, 0, s, B, F, k, ids, (const float*)table,
                       (bf16_t*)xbuf, ldx);
  else
    hipLaunchKernelGGL((gather_x_kernel<float, float>), grid, blk, 0, s, B, F, k, ids, (const float*)table,
                       (float*)xbuf, ldx);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
