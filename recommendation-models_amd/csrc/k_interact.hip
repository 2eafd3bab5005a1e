// k_interact.hip -- DCN cross network and PNN inner-product encoder (gfx950).
//
// DCN  model/dcn/CrossEncoder.scala:40-55, 107-152:
//   x_{l+1} = ((x0 * (w_l . x_l)) + x_l) + beta_l   (Linear(D->1, no bias), MM, CAddTable, CAdd(1))
//   the x_L slice of the output Linear (:176-185) is folded in: pre2[b] = x_L . W_out[0:D].
//   One wave per sample; x0 / x_l live in registers (D <= 1024 -> <= 16 per lane).
// PNN  model/pnn/ProductEncoder.scala:84-120, bnn/Gather.scala:19-47, bnn/DotProduct2.scala:16-26:
//   ip[b,p] = sum_t e[b,i_p,t] * e[b,j_p,t] over pairs (i < j) in lexicographic order;
//   writes the row [x | ip] (zero padded) that feeds ONE GEMM for Wz x + Wp ip (K = D + P).
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

int launch_cross(hipStream_t s, int B, int F, int k, int L, const int32_t* ids, const void* table, int dt,
                 const float* cross_w, const float* cross_b, const float* wo_x, float* pre2) {
  if (B <= 0) return RMX_OK;
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

int launch_product(hipStream_t s, int B, int F, int k, const int32_t* ids, const void* table, int dt,
                   const int32_t* pairs, int P, void* xbuf, int xdt, int ldx) {
  if (B <= 0) return RMX_OK;
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
