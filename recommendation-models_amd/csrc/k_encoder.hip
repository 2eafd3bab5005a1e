// k_encoder.hip -- HBM-bound encoder kernels: embedding / first-order gather, Scatter
// first order, FM second order, plus the synthetic id / table generators.
//
//   gather        yr/model/ParRecModel.scala:279-306 (makeWeights / makeEmbeddings)
//   first order   bnn/Scatter.scala:17-36 (ascending-n accumulation into row index[n])
//   FM            yr/model/encoder/SecondOrderEncoder.scala:19-34
//                 y2 = 0.5 * (sum_j[(sum_f e)^2 - sum_f e^2] / k)
//
// The FM / first-order sums follow the oracle's order exactly (sequential over f, then
// sequential over j) with FMA contraction disabled, so y1 and y2 are bit-identical to
// oracle/rmx_oracle.c.
#include "rmx_internal.hpp"

namespace rmx {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// mode: 0 = y = y1 (first order), 1 = y = y1 + y2 (DeepFM), 2 = prob = sigmoid(y1 + beta) (LR),
//       3 = y += y2 (L-A path with an irregular COO index: y already holds y1 from the CSR kernel).
// k = 16 fast path: 4 lanes per sample (one float4 of the 64-B row each), 16 samples per wave,
// all F row loads of a lane independent (ids staged in registers first).
// xo (nullable, MODE 0 / 1 / 3): also store the gathered rows as the fp32 x = [B][F * 16] (row stride F * 16):
// the training forward's tower input, written from the same loads (float4 per lane, 64 B per field)
template <int MODE, class T>
__global__ __launch_bounds__(256) void encoder_k16_kernel(int M, const int32_t* __restrict__ ids,
                                                          const T* __restrict__ table,
                                                          const T* __restrict__ wtab, int F,
                                                          float* __restrict__ y, float beta,
                                                          float* __restrict__ prob, int ld, int wld,
                                                          float* __restrict__ xo, float* __restrict__ so) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int s = lane >> 2, c = lane & 3;
  const int b = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + s;
  const bool valid = b < M;
  const int bb = valid ? b : 0;
  constexpr bool FM = MODE == 1 || MODE == 3;
  const bool rows = FM || (MODE == 0 && xo != nullptr);  // the rows are loaded
  float4* xr = xo && valid ? reinterpret_cast<float4*>(xo + (int64_t)b * F * 16) + c : nullptr;
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f), q4 = s4;
  float y1 = 0.f;
  int f = 0;
  for (; f + 8 <= F; f += 8) {
    int id[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) id[u] = ids ? ids[(int64_t)bb * F + f + u] : bb * F + f + u;
    float4 v[8];
    float wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (rows) v[u] = load4(table + (int64_t)id[u] * ld + c * 4);
      if (MODE != 3) wv[u] = (c == 0) ? ld1(wtab + (int64_t)id[u] * wld) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (FM) {
        s4.x += v[u].x; s4.y += v[u].y; s4.z += v[u].z; s4.w += v[u].w;
        q4.x += v[u].x * v[u].x; q4.y += v[u].y * v[u].y;
        q4.z += v[u].z * v[u].z; q4.w += v[u].w * v[u].w;
      }
      if (MODE != 3) y1 += wv[u];
      if (xr) xr[(f + u) * 4] = v[u];
    }
  }
  for (; f < F; ++f) {
    const int id = ids ? ids[(int64_t)bb * F + f] : bb * F + f;
    if (rows) {
      const float4 v = load4(table + (int64_t)id * ld + c * 4);
      if (FM) {
        s4.x += v.x; s4.y += v.y; s4.z += v.z; s4.w += v.w;
        q4.x += v.x * v.x; q4.y += v.y * v.y; q4.z += v.z * v.z; q4.w += v.w * v.w;
      }
      if (xr) xr[f * 4] = v;
    }
    if (MODE != 3 && c == 0) y1 += ld1(wtab + (int64_t)id * wld);
  }
  // so (nullable, FM modes): the FM sums s_j = sum_f e_fj (field order from 0) as [B][16], read by the
  // training backward's fused embedding gradient (k_gemm.hpp store_rows, emb_grad_kernel's s)
  if (FM && so && valid) reinterpret_cast<float4*>(so + (int64_t)b * 16)[c] = s4;
  float y2 = 0.f;
  if (MODE == 1 || MODE == 3) {
    // d_j = s_j^2 - q_j for j = 4c..4c+3; lane c==0 sums j = 0..15 sequentially.
    float d0 = s4.x * s4.x - q4.x, d1 = s4.y * s4.y - q4.y;
    float d2 = s4.z * s4.z - q4.z, d3 = s4.w * s4.w - q4.w;
    float acc = 0.f;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int src = (lane & ~3) | cc;
      acc += __shfl(d0, src);
      acc += __shfl(d1, src);
      acc += __shfl(d2, src);
      acc += __shfl(d3, src);
    }
    y2 = 0.5f * (acc / 16.0f);
  }
  if (!valid || c != 0) return;
  if (MODE == 0) y[b] = y1;
  if (MODE == 1) y[b] = y1 + y2;
  if (MODE == 2) prob[b] = 1.0f / (1.0f + expf(-(y1 + beta)));
  if (MODE == 3) y[b] = y[b] + y2;  // y holds y1 from the CSR kernel
}

// Round 5: the same lane layout and arithmetic (y1 + y2 bit-identical to encoder_k16_kernel), with fewer
// dependent round trips to memory.  The kernel above loads 8 ids, then their 8 rows, then the next 8 ids:
// 10 round trips for F = 39, each exposed (B = 65,536 gives only 16 waves per CU, so nothing else hides
// them; V = 100M row table: 0.106 ms, 0.78 of the 128-B line rate of HBM).  Here the 4 lanes of a sample
// load the sample's ids of a 40-field chunk once, coalesced (lane c: fields 4i + c), share them with a quad
// DPP broadcast, and request the rows (+ first-order weights) in batches of U: 1 + ceil(F / U) round trips.
// Modes 0, 1, 2 with ids given; XO: also the training forward's outputs (x, and the FM sums in mode 1) from the
// same loads, as encoder_k16_kernel writes them (mode 3 and the implicit-id L-A path keep the kernel above).
__device__ __attribute__((aligned(16))) float g_enc_zero16[16];  // the zero row of fields past F

template <int J>
__device__ __forceinline__ int quad_bcast(int v) {  // every lane of a quad takes the quad's lane J
  return __builtin_amdgcn_mov_dpp(v, J * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ int quad_bcast(int v, int j) {  // (j is a constant after unrolling)
  switch (j) {
    case 0: return quad_bcast<0>(v);
    case 1: return quad_bcast<1>(v);
    case 2: return quad_bcast<2>(v);
    default: return quad_bcast<3>(v);
  }
}

template <int MODE, class T, int U, bool XO = false>
__global__ __launch_bounds__(256) void encoder_k16v2_kernel(int M, const int32_t* __restrict__ ids,
                                                            const T* __restrict__ table,
                                                            const T* __restrict__ wtab, int F,
                                                            float* __restrict__ y, float beta,
                                                            float* __restrict__ prob, int ld, int wld,
                                                            float* __restrict__ xo = nullptr,
                                                            float* __restrict__ so = nullptr) {
#pragma clang fp contract(off)
  constexpr int NI = 10, CH = 4 * NI;  // ids per lane / fields per chunk
  constexpr int NB = (CH + U - 1) / U;
  constexpr bool FM = MODE == 1;
  constexpr bool ROWS = FM || (XO && MODE == 0);
  const int lane = threadIdx.x & 63;
  const int s = lane >> 2, c = lane & 3;
  const int b = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + s;
  const bool valid = b < M;
  const int32_t* irow = ids + (int64_t)(valid ? b : 0) * F;
  float4* xr = XO && xo && valid ? reinterpret_cast<float4*>(xo + (int64_t)b * F * 16) + c : nullptr;  // (xo nullable)
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f), q4 = s4;
  float y1 = 0.f;
  // branch-free inside a batch (a per-lane or per-field branch around a load made the compiler wait for each
  // load before the next): every lane loads every id / row / weight; a field past F reads a zero row and a
  // zero weight (x + 0 = x: the sums keep their bits), whose address is selected, not branched to
  const float* zero16 = g_enc_zero16;
  for (int f0 = 0; f0 < F; f0 += CH) {
    int idv[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int f = f0 + 4 * i + c;
      idv[i] = irow[f < F ? f : F - 1];
    }
#pragma unroll
    for (int h = 0; h < NB; ++h) {
      if (f0 + h * U >= F) break;  // (wave-uniform, per batch)
      float4 v[U];
      float wv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int uu = h * U + u;
        if (uu >= CH) break;  // (compile time)
        // field f0 + uu: its id is lane (s, uu & 3)'s idv[uu >> 2] -- a quad_perm(j, j, j, j) broadcast
        const int id = quad_bcast(idv[uu >> 2], uu & 3);
        const bool live = f0 + uu < F;
        const T* rsrc = live ? table + (int64_t)id * ld + c * 4 : reinterpret_cast<const T*>(zero16);
        const T* wsrc = live ? wtab + (int64_t)id * wld : reinterpret_cast<const T*>(zero16);
        if (ROWS) v[u] = load4(rsrc);
        wv[u] = ld1(wsrc);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (h * U + u >= CH) break;
        if (FM) {
          s4.x += v[u].x; s4.y += v[u].y; s4.z += v[u].z; s4.w += v[u].w;
          q4.x += v[u].x * v[u].x; q4.y += v[u].y * v[u].y;
          q4.z += v[u].z * v[u].z; q4.w += v[u].w * v[u].w;
        }
        y1 += wv[u];
      }
      if constexpr (XO) {  // after the batch's sums: the stores wait for nothing the sums did not
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int uu = h * U + u;
          if (uu >= CH) break;
          if (xr && f0 + uu < F) xr[(f0 + uu) * 4] = v[u];
        }
      }
    }
  }
  if (XO && FM && so && valid) reinterpret_cast<float4*>(so + (int64_t)b * 16)[c] = s4;
  float y2 = 0.f;
  if (FM) {  // encoder_k16_kernel's reduction, the same order
    float d0 = s4.x * s4.x - q4.x, d1 = s4.y * s4.y - q4.y;
    float d2 = s4.z * s4.z - q4.z, d3 = s4.w * s4.w - q4.w;
    float acc = 0.f;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int src = (lane & ~3) | cc;
      acc += __shfl(d0, src);
      acc += __shfl(d1, src);
      acc += __shfl(d2, src);
      acc += __shfl(d3, src);
    }
    y2 = 0.5f * (acc / 16.0f);
  }
  if (!valid || c != 0) return;
  if (MODE == 0) y[b] = y1;
  if (MODE == 1) y[b] = y1 + y2;
  if (MODE == 2) prob[b] = 1.0f / (1.0f + expf(-(y1 + beta)));
}

// Generic-k fallback: one thread per sample, oracle order.
template <int MODE, class T>
__global__ __launch_bounds__(256) void encoder_generic_kernel(int M, const int32_t* __restrict__ ids,
                                                              const T* __restrict__ table,
                                                              const T* __restrict__ wtab, int F,
                                                              int k, float* __restrict__ y,
                                                              float beta, float* __restrict__ prob, int ld,
                                                              int wld) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= M) return;
  float y1 = 0.f, y2 = 0.f;
  if (MODE != 3)
    for (int f = 0; f < F; ++f) {
      const int id = ids ? ids[(int64_t)b * F + f] : b * F + f;
      y1 += ld1(wtab + (int64_t)id * wld);
    }
  if (MODE == 1 || MODE == 3) {
    float acc = 0.f;
    for (int j = 0; j < k; ++j) {
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const int id = ids ? ids[(int64_t)b * F + f] : b * F + f;
        const float v = ld1(table + (int64_t)id * ld + j);
        s += v;
        q += v * v;
      }
      acc += s * s - q;
    }
    y2 = 0.5f * (acc / (float)k);
  }
  if (MODE == 0) y[b] = y1;
  if (MODE == 1) y[b] = y1 + y2;
  if (MODE == 2) prob[b] = 1.0f / (1.0f + expf(-(y1 + beta)));
  if (MODE == 3) y[b] = y[b] + y2;
}

template <class T>
static void encoder_launch_t(hipStream_t s, int mode, int M, const int32_t* ids, const T* table, const T* wtab, int F,
                             int k, float* y, float bt, float* prob, int ld, int wld, float* xo, float* so) {
  // knob "enc_u" (round 5): rows per batch of the v2 kernel, 0 = the kernel above
  const int eu = tuning_get("enc_u", 20);
  // (x / FM sums for the training forward: knob "enc_v2_x", default 1)
  const bool xs = xo || so;
  if ((k == 16 || mode == 2) && ids && mode != 3 && (eu == 13 || eu == 20) &&
      (!xs || (mode != 2 && eu == 20 && tuning_get("enc_v2_x", 1) != 0))) {
    dim3 grid((M + 63) / 64);
    if (xs) {
      if (mode == 0)
        hipLaunchKernelGGL((encoder_k16v2_kernel<0, T, 20, true>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt,
                           prob, ld, wld, xo, so);
      else
        hipLaunchKernelGGL((encoder_k16v2_kernel<1, T, 20, true>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt,
                           prob, ld, wld, xo, so);
      return;
    }
#define RMX_ENC2(MD, UU) hipLaunchKernelGGL((encoder_k16v2_kernel<MD, T, UU>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt, prob, ld, wld)
    if (eu == 13) {
      if (mode == 0) RMX_ENC2(0, 13); else if (mode == 1) RMX_ENC2(1, 13); else RMX_ENC2(2, 13);
    } else {
      if (mode == 0) RMX_ENC2(0, 20); else if (mode == 1) RMX_ENC2(1, 20); else RMX_ENC2(2, 20);
    }
#undef RMX_ENC2
    return;
  }
  if (k == 16 || mode == 2) {  // LR (mode 2) never reads the table: any k takes the 4-lane path
    dim3 grid((M + 63) / 64);
    switch (mode) {
      case 0: hipLaunchKernelGGL((encoder_k16_kernel<0, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt, prob, ld, wld, xo, so); break;
      case 1: hipLaunchKernelGGL((encoder_k16_kernel<1, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt, prob, ld, wld, xo, so); break;
      case 2: hipLaunchKernelGGL((encoder_k16_kernel<2, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt, prob, ld, wld, nullptr, nullptr); break;
      default: hipLaunchKernelGGL((encoder_k16_kernel<3, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, y, bt, prob, ld, wld, xo, so); break;
    }
  } else {
    dim3 grid((M + 255) / 256);
    switch (mode) {
      case 0: hipLaunchKernelGGL((encoder_generic_kernel<0, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, k, y, bt, prob, ld, wld); break;
      case 1: hipLaunchKernelGGL((encoder_generic_kernel<1, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, k, y, bt, prob, ld, wld); break;
      default: hipLaunchKernelGGL((encoder_generic_kernel<3, T>), grid, dim3(256), 0, s, M, ids, table, wtab, F, k, y, bt, prob, ld, wld); break;
    }
  }
}

int launch_encoder(hipStream_t s, int mode, int M, const int32_t* ids, const void* table, const void* wtab, int dt,
                   int F, int k, float* y, const float* beta, float* prob, int ld, int wld, float* xo, float* so) {
  if (M <= 0) return RMX_OK;
  if (so && (k != 16 || (mode != 1 && mode != 3))) {
    set_error("encoder: the FM-sum output needs k = 16 and an FM mode");
    return RMX_E_INVALID;
  }
  if (xo && (k != 16 || mode == 2)) {
    set_error("encoder: the gathered-row output needs k = 16 and a table-reading mode");
    return RMX_E_INVALID;
  }
  const float bt = beta ? *beta : 0.f;
  ld = ld > 0 ? ld : (k == 16 || mode == 2 ? 16 : k);
  wld = wld > 0 ? wld : 1;
  if (dt == kBF16)
    encoder_launch_t(s, mode, M, ids, (const bf16_t*)table, (const bf16_t*)wtab, F, k, y, bt, prob, ld, wld, xo, so);
  else
    encoder_launch_t(s, mode, M, ids, (const float*)table, (const float*)wtab, F, k, y, bt, prob, ld, wld, xo, so);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// Scatter first order over a CSR view of a (row-sorted) COO index: y[b] = sum of w[n] for
// n in [row_ptr[b], row_ptr[b+1]) in ascending n (bnn/Scatter.scala:25-33 order).
__global__ __launch_bounds__(256) void first_order_csr_kernel(int B, const int64_t* __restrict__ row_ptr,
                                                              const float* __restrict__ w,
                                                              float* __restrict__ y) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;
  for (int64_t n = row_ptr[b]; n < row_ptr[b + 1]; ++n) acc += w[n];
  y[b] = acc;
}

int launch_first_order_csr(hipStream_t s, int B, const int64_t* row_ptr, const float* w, float* y) {
  if (B <= 0) return RMX_OK;
  hipLaunchKernelGGL(first_order_csr_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, row_ptr, w, y);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

__global__ void sigmoid_out_kernel(int B, const float* __restrict__ y, float beta, float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = 1.0f / (1.0f + expf(-(y[b] + beta)));
}

int launch_sigmoid_out(hipStream_t s, int B, const float* y, float beta, float* out) {
  if (B <= 0) return RMX_OK;
  hipLaunchKernelGGL(sigmoid_out_kernel, dim3((B + 255) / 256), dim3(256), 0, s, B, y, beta, out);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// ----------------------------------------------------------- synthetic ------
__global__ void gen_ids_kernel(uint64_t seed, int64_t row0, int B, int F, uint64_t per, int32_t* ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * F) return;
  const int64_t b = i / F;
  const int f = (int)(i - b * F);
  const uint64_t cnt = (uint64_t)(row0 + b) * (uint64_t)F + (uint64_t)f;
  ids[i] = (int32_t)((uint64_t)f * per + splitmix64(seed ^ cnt) % per);
}

// Zipf-like ids (SURVEY.md §8d secondary distribution): rank r in field f with P(r) ~ (r+1)^-s,
// drawn by inverting the continuous power law on [1, per + 1) in double precision.
__global__ void gen_ids_zipf_kernel(uint64_t seed, int64_t row0, int B, int F, uint64_t per, double a, double span,
                                    int32_t* ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * F) return;
  const int64_t b = i / F;
  const int f = (int)(i - b * F);
  const uint64_t cnt = (uint64_t)(row0 + b) * (uint64_t)F + (uint64_t)f;
  const double u = (double)(splitmix64(seed ^ cnt) >> 11) * 0x1.0p-53;
  int64_t r = (int64_t)floor(pow(1.0 + u * span, 1.0 / a)) - 1;
  r = r < 0 ? 0 : (r >= (int64_t)per ? (int64_t)per - 1 : r);
  ids[i] = (int32_t)((uint64_t)f * per + (uint64_t)r);
}

int launch_gen_ids_zipf(hipStream_t s, uint64_t seed, int64_t row0, int B, int F, int64_t V, double zs,
                        int32_t* ids) {
  const int64_t n = (int64_t)B * F;
  if (n <= 0) return RMX_OK;
  const uint64_t per = (uint64_t)(V / F);
  const double a = 1.0 - zs;
  const double span = pow((double)per + 1.0, a) - 1.0;
  hipLaunchKernelGGL(gen_ids_zipf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seed, row0, B, F, per,
                     a, span, ids);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

int launch_gen_ids(hipStream_t s, uint64_t seed, int64_t row0, int B, int F, int64_t V, int32_t* ids) {
  const int64_t n = (int64_t)B * F;
  if (n <= 0) return RMX_OK;
  hipLaunchKernelGGL(gen_ids_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seed, row0, B,
                     F, (uint64_t)(V / F), ids);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// [V][32] line copy of a k = 16 table: row i = [emb[i][0..16) | w[i] | 15 zeros] (rmx_table::line): one 128-B
// memory line per id for fp32, one 64-B half line for bf16.  One lane per 16-B piece (8 fp32 / 4 bf16 lanes
// per row, coalesced rows).
template <class T>
__global__ __launch_bounds__(256) void pack_lines_kernel(int64_t V, const T* __restrict__ emb, const T* __restrict__ w,
                                                        T* __restrict__ line) {
  constexpr int E = 16 / sizeof(T);  // elements per 16-B piece
  constexpr int P = 32 / E;          // pieces per line row
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / P;
  const int c = (int)(t - i * P);
  if (i >= V) return;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < 16 / E) {
    v = reinterpret_cast<const float4*>(emb + i * 16)[c];
  } else if (c == 16 / E) {
    T* e = reinterpret_cast<T*>(&v);
    e[0] = w[i];
  }
  reinterpret_cast<float4*>(line + i * 32)[c] = v;
}

int launch_pack_lines(hipStream_t s, int64_t V, const void* emb, const void* w, void* line, int dt) {
  if (V <= 0) return RMX_OK;
  if (dt == kBF16)
    hipLaunchKernelGGL(pack_lines_kernel<bf16_t>, dim3((unsigned)((V * 4 + 255) / 256)), dim3(256), 0, s, V,
                       (const bf16_t*)emb, (const bf16_t*)w, (bf16_t*)line);
  else
    hipLaunchKernelGGL(pack_lines_kernel<float>, dim3((unsigned)((V * 8 + 255) / 256)), dim3(256), 0, s, V,
                       (const float*)emb, (const float*)w, (float*)line);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <class T>
__global__ void fill_table_kernel(uint64_t seed, int64_t V, int k, float scale, T* w, T* emb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = V * (k + 1);
  if (i >= tot) return;
  const int64_t id = i / (k + 1);
  const int j = (int)(i - id * (k + 1));
  const uint64_t h = splitmix64(seed ^ (uint64_t)i);  // i == id*(k+1) + j
  const float v = (float)((int32_t)(h >> 40) - 8388608) * scale;
  if (j < k) st1(emb + id * k + j, v);
  else st1(w + id, v);
}

int launch_fill_table(hipStream_t s, uint64_t seed, int64_t V, int k, void* w, void* emb, int dt) {
  const int64_t tot = V * (k + 1);
  const float scale = 0.05f * (1.0f / 8388608.0f);
  if (dt == kBF16)
    hipLaunchKernelGGL(fill_table_kernel<bf16_t>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, seed, V, k,
                       scale, (bf16_t*)w, (bf16_t*)emb);
  else
    hipLaunchKernelGGL(fill_table_kernel<float>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, seed, V, k,
                       scale, (float*)w, (float*)emb);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

template <class T>
__global__ void gather_kernel(int64_t n, const int32_t* __restrict__ ids, const T* __restrict__ wtab,
                              const T* __restrict__ emb, int k, float* __restrict__ w_out, float* __restrict__ e_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * (k + 1)) return;
  const int64_t r = i / (k + 1);
  const int j = (int)(i - r * (k + 1));
  const int id = ids[r];
  if (j < k) {
    if (e_out) e_out[r * k + j] = ld1(emb + (int64_t)id * k + j);
  } else if (w_out) {
    w_out[r] = ld1(wtab + id);
  }
}

int launch_gather(hipStream_t s, int64_t n, const int32_t* ids, const void* wtab, const void* emb, int dt, int k,
                  float* w_out, float* e_out) {
  if (n <= 0) return RMX_OK;
  const int64_t tot = n * (k + 1);
  if (dt == kBF16)
    hipLaunchKernelGGL(gather_kernel<bf16_t>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, n, ids,
                       (const bf16_t*)wtab, (const bf16_t*)emb, k, w_out, e_out);
  else
    hipLaunchKernelGGL(gather_kernel<float>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, n, ids,
                       (const float*)wtab, (const float*)emb, k, w_out, e_out);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

__global__ void convert_bf16_kernel(const float* __restrict__ src, int64_t n, bf16_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (bf16_t)src[i];
}

__global__ void widen_bf16_kernel(const bf16_t* __restrict__ src, int64_t n, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

int launch_widen_bf16(hipStream_t s, const bf16_t* src, int64_t n, float* dst) {
  if (n <= 0) return RMX_OK;
  hipLaunchKernelGGL(widen_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, n, dst);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

int launch_convert_bf16(hipStream_t s, const float* src, int64_t n, bf16_t* dst) {
  if (n <= 0) return RMX_OK;
  hipLaunchKernelGGL(convert_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, n, dst);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// W (out x in row-major at mats + w_off) -> [Kpad/16][Npad][16]; bias -> [Npad].
// (PNN: columns >= K1 come from a second matrix at w_off2; bias_mode 2 broadcasts one scalar.)
// value of W[n][kx] of a packed layer (PNN: two matrices side by side; DCN: extra cross rows)
__device__ __forceinline__ float layer_w(const float* __restrict__ mats, const DenseLayer& L, int n, int kx) {
  if (n >= L.N || kx >= L.K) return 0.f;
  if (L.N1 >= 0 && n >= L.N1) {
    const int e = n - L.N1;
    return e < L.nx ? mats[L.w_off_x + (int64_t)e * L.K + kx] : mats[L.w_off_o + kx];
  }
  if (L.K1 < 0) return mats[L.w_off + (int64_t)n * L.K + kx];
  if (kx < L.K1) return mats[L.w_off + (int64_t)n * L.K1 + kx];
  return mats[L.w_off2 + (int64_t)n * (L.K - L.K1) + (kx - L.K1)];
}

__global__ void pack_linear_kernel(const float* __restrict__ mats, DenseLayer L, int64_t b_off, int bias_mode,
                                   int K, int N, int Kpad, int Npad, float* __restrict__ Wp, float* __restrict__ bp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)Kpad * Npad;
  if (i < tot) {
    const int kk = (int)(i & 15);
    const int64_t rest = i >> 4;
    const int n = (int)(rest % Npad);
    const int c = (int)(rest / Npad);
    const int kx = c * 16 + kk;
    Wp[i] = layer_w(mats, L, n, kx);
  }
  if (i < Npad) {
    const int nb = L.N1 >= 0 ? L.N1 : N;  // extra DCN rows have no bias
    float v = 0.f;
    if (i < nb && bias_mode == 1) v = mats[b_off + i];
    if (i < nb && bias_mode == 2) v = mats[b_off];
    bp[i] = v;
  }
}

// bf16 packing: [Kpad/32][Npad][32] (one 64-B row = 32 bf16 of one output column), RNE rounding
__global__ void pack_linear_bf16_kernel(const float* __restrict__ mats, DenseLayer L, int Kpad, int Npad,
                                        bf16_t* __restrict__ Wp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)Kpad * Npad;
  if (i >= tot) return;
  const int kk = (int)(i & 31);
  const int64_t rest = i >> 5;
  const int n = (int)(rest % Npad);
  const int c = (int)(rest / Npad);
  const int kx = c * 32 + kk;
  const float v = layer_w(mats, L, n, kx);
  Wp[i] = (bf16_t)v;
}

int launch_pack_linear(hipStream_t s, const float* mats_dev, DenseLayer& L) {
  const int64_t tot = (int64_t)L.Kpad * L.Npad;
  const int64_t n = tot > L.Npad ? tot : L.Npad;
  // bias (and, for fp32 layers, W)
  hipLaunchKernelGGL(pack_linear_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, mats_dev, L,
                     L.b_off, L.b_off >= 0 ? L.bias_mode : 0, L.K, L.N, L.W16 ? 0 : L.Kpad, L.Npad, L.W, L.b);
  RMX_HIP(hipGetLastError());
  if (L.W16) {
    hipLaunchKernelGGL(pack_linear_bf16_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, mats_dev, L,
                       L.Kpad, L.Npad, L.W16);
    RMX_HIP(hipGetLastError());
  }
  return RMX_OK;
}

template <class T>
__global__ void transpose_kmajor_kernel(const float* __restrict__ src, int64_t V, int k, T* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V * k) return;
  const int64_t id = i / k;
  const int j = (int)(i - id * k);
  st1(dst + i, src[(int64_t)j * V + id]);
}

int launch_transpose_kmajor(hipStream_t s, const float* src_kv, int64_t V, int k, void* dst_vk, int dt) {
  const int64_t tot = V * k;
  if (tot <= 0) return RMX_OK;
  if (dt == kBF16)
    hipLaunchKernelGGL(transpose_kmajor_kernel<bf16_t>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src_kv,
                       V, k, (bf16_t*)dst_vk);
  else
    hipLaunchKernelGGL(transpose_kmajor_kernel<float>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src_kv,
                       V, k, (float*)dst_vk);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

}  // namespace rmx
