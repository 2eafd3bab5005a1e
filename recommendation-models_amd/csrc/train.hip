// train.hip -- RecModel.backward on the device: BCE loss + the gradients the reference writes
// back into the caller's arrays.
//
// Reference: yr/model/deepfm/DeepFM.scala:83-124 (and the other models' backward halves),
// bnn/Scatter.scala:38-59, yr/util/GradUtil.scala:7-42, yr/util/BackwardUtil.scala:6-30
// (paths under /root/reference/src/main/scala/, yr/ = io/yaochi/recommendation/,
// bnn/ = com/intel/analytics/bigdl/nn/).  BigDL BCECriterion (sizeAverage, eps = 1e-12) and
// Sigmoid backward as published (oracle/rmx_oracle_train.c states the math).
//
// Pass structure (fp32, one stream):
//   forward   same kernels as the inference path, but every hidden activation h_l [B][Npad_l]
//             is stored (ReLU-store epilogue), the tower input x = Reshape(E) is materialised,
//             and the logit head runs over the stored last hidden layer;
//   loss      bce_kernel: p -> dL/dz per row + per-block partial sums (deterministic tree);
//   tower     per layer, from the top: dW = dPre^T x_in (wgrad_s3_kernel, split GEMM) and dx_in =
//             dPre W (the forward's split GEMM on W^T planes, ReLU mask of the layer below fused;
//             gemm_f32_kernel for layers without W^T planes), db = dPre^T 1 (GEMV);
//   CIN       dC_l = gpre^T z (wgrad), dL/dz = gpre C_l (split GEMM on C_l^T planes), contracted
//             into dL/dx0 and dL/du_{l-1}; DCN cross GEMMs on gemm_f32_kernel (no library GEMM);
//   encoders  emb_grad_kernel: dL/dE = dx (tower) + FM term dz (s_j - e_fj) / k; dL/dw[n] =
//             dz[index[n]] (Scatter backward).
#include <algorithm>
#include <type_traits>
#ifndef RMX_WGRAD_SQ_DIAG
#define RMX_WGRAD_SQ_DIAG 0  // 1: the wgrad_sq timing probes (knob wgrad_diag) are built
#endif
#include <vector>

#include "rmx_models.hpp"

namespace rmx {

struct TrainState {
  int B = 0;
  int ldx = 0;                  // row stride of x / dx
  float* x = nullptr;           // [B][ldx] tower input (Reshape(B, F*k) of the gathered rows)
  std::vector<float*> h;        // per tower layer [B][Npad]
  std::vector<float*> hm;       // per tower layer [B][16] ReLU mask bits (uint32), written by the row-owner
  std::vector<char> hm_ok;      //   forward kernels this step (k_layer_s3.hip / k_head_s3.hip XS); hm_ok: valid
  float* g[2] = {nullptr, nullptr};  // [B][maxld] dPre / dx ping-pong
  float* p = nullptr;           // [B] probabilities
  float* dz = nullptr;          // [B] dL/dlogit
  float* ones = nullptr;        // [B]
  double* part = nullptr;       // [2 * kMaxParts] loss / dz partial sums
  // DCN (cross stack in closed form, k_interact.hip cross_finish_kernel)
  float* xcol = nullptr;        // [B][L + 1] u_l = w_l . x0, v = W_out[0:D] . x0
  float* wc = nullptr;          // [L + 1][D] rows w_0 .. w_{L-1}, W_out[0:D]
  float* coef = nullptr;        // [B][L + 1] x0-coefficients of the cross gradients
  float* cst = nullptr;         // [B][2L + 1] per-row constants (see cross_back_kernel)
  float* gwc = nullptr;         // [L + 1][D] gradient of wc before the constant parts
  float* tmp = nullptr;         // [max(Npad, 2L + 1)] column sums
  // xDeepFM CIN (rows r = b*k + j, R = B*k)
  std::vector<float*> u;        // [R][Npad_l] maps of every CIN layer
  float* x0 = nullptr;          // [R][F] x0[b*k + j][f] = e[b][f][j]
  float* gx0 = nullptr;         // [R][F] dL/dx0 (CIN part)
  float* gu[2] = {nullptr, nullptr};  // [R][maxNpad] dL/du of the layer below (from the layer above)
  float* gpre = nullptr;        // [R][maxNpad] dL/d(pre-activation) of the current layer
  float* dzr = nullptr;         // [R] dz[r / k]
  float* zb = nullptr;          // [rc][max F*Hp] Z = x0 (x) u_prev chunk, then its gradient
  float* onesR = nullptr;       // [R]
  int rc = 0;                   // rows per chunk (a multiple of k)
  float* part2 = nullptr;       // [cap_part] slice partials of wgrad / colsum
  int64_t cap_part = 0;
  float* fms = nullptr;         // DeepFM, k = 16: [B][16] FM sums s_j of the forward (fused embedding gradient)
  bool fms_valid = false;       // this step's forward wrote fms
};

namespace {

constexpr int kRedThreads = 256, kMaxParts = 1024;

template <class T>
void tfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

int talloc(float** p, size_t n) {
  if (hipMalloc((void**)p, sizeof(float) * std::max<size_t>(n, 1)) != hipSuccess) {
    set_error("backward: out of device memory (" + std::to_string(n * sizeof(float)) + " bytes)");
    return RMX_E_NOMEM;
  }
  return RMX_OK;
}

__global__ void fill_kernel(int n, float v, float* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = v;
}

// BCECriterion + Sigmoid backward, per row; block partial sums of the loss terms and of dz.
__global__ __launch_bounds__(kRedThreads) void bce_kernel(int B, const float* __restrict__ p,
                                                          const float* __restrict__ targets, float* __restrict__ dz,
                                                          int per_block, double* __restrict__ part) {
  __shared__ double sl[kRedThreads], sg[kRedThreads];
  const float eps = 1e-12f, norm = 1.0f / (float)B;
  double l = 0.0, gsum = 0.0;
  const int b0 = blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  for (int b = b0 + threadIdx.x; b < b1; b += kRedThreads) {
    const float x = p[b];
    const float t = targets[b] > 0.f ? 1.f : 0.f;  // DeepFM.scala:106
    l += -((double)t * log((double)x + eps) + (1.0 - t) * log(1.0 - (double)x + eps));
    const float gp = -(t - x) * norm / ((1.f - x + eps) * (x + eps));  // dL/dp
    const float g = gp * (1.f - x) * x;                                 // Sigmoid backward
    dz[b] = g;
    gsum += g;
  }
  sl[threadIdx.x] = l;
  sg[threadIdx.x] = gsum;
  __syncthreads();
  for (int o = kRedThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sl[threadIdx.x] += sl[threadIdx.x + o];
      sg[threadIdx.x] += sg[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x] = sl[0];
    part[kMaxParts + blockIdx.x] = sg[0];
  }
}

// loss = sum(part_l) / B; every non-null target of the bias gradient = sum(part_g).  256 threads: thread t
// sums parts t, t + 256, ... in order, then a fixed tree (one thread over 1,024 parts was a chain of
// dependent L2 loads: ~0.1 ms)
__global__ __launch_bounds__(256) void bce_finish_kernel(int nparts, int B, const double* __restrict__ part,
                                                         float* __restrict__ loss, float* __restrict__ gbias,
                                                         float* __restrict__ gbias2) {
  __shared__ double sl[256], sg[256];
  double l = 0.0, g = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    l += part[i];
    g += part[kMaxParts + i];
  }
  sl[threadIdx.x] = l;
  sg[threadIdx.x] = g;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sl[threadIdx.x] += sl[threadIdx.x + o];
      sg[threadIdx.x] += sg[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  if (loss) *loss = (float)(sl[0] / B);
  if (gbias) *gbias = (float)sg[0];
  if (gbias2) *gbias2 = (float)sg[0];
}

// The training head in one pass over the last hidden activations h (knob "train_head_fused", default
// on): per row (one wave), the logit and p exactly as tower_head_kernel (same products, same order:
// bitwise the same p), BigDL BCECriterion + Sigmoid backward as bce_kernel (dz = dL/dlogit), the output
// layer's dPre = dz * wo masked by ReLU (h > 0) as head_back4_kernel, and per-block partial sums of the
// loss, of dz (bias gradients) and of dz * h[:, n] (dW_out, reduced over blocks by slice_reduce_kernel).
// One read of h instead of three (tower_head, head_back, colsum) and no launches in between:
// DeepFM B = 65,536: tower_head + bce + head_back 0.036 + 0.024 + 0.085 ms.
constexpr int kHeadCols = 8;  // columns per lane: N <= 512
__global__ __launch_bounds__(256) void head_train_kernel(int B, int N, const float* __restrict__ h, int ldh, OutArgs oa,
                                                         const float* __restrict__ targets, float* __restrict__ dz,
                                                         float* __restrict__ g, int ldg, int per_block,
                                                         double* __restrict__ part, float* __restrict__ cpart) {
  __shared__ double sl[4], sg[4];
  __shared__ float cs[4][kHeadCols * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float eps = 1e-12f, norm = 1.0f / (float)B;
  const int b0 = blockIdx.x * per_block, b1 = min(B, b0 + per_block);
  float col[kHeadCols];
#pragma unroll
  for (int q = 0; q < kHeadCols; ++q) col[q] = 0.f;
  double l = 0.0, gsum = 0.0;
  // the BCE loss terms (two fp64 logs per row) run 64 rows at a time, one row per lane: row i of the
  // wave parks its p / target in lane i & 63 (computed by one lane per row inside the row loop they cost
  // ~1.5 k cycles of the whole wave's issue per row)
  float px = 0.5f, pt = 0.f;
  int npend = 0;
  auto flush = [&]() {
    if (lane < npend) l += -((double)pt * log((double)px + eps) + (1.0 - pt) * log(1.0 - (double)px + eps));
    npend = 0;
  };
  float wv4[kHeadCols];
#pragma unroll
  for (int q = 0; q < kHeadCols; ++q) wv4[q] = lane + 64 * q < N ? oa.wo[lane + 64 * q] : 0.f;
  // the wave's rows b0 + wv, b0 + wv + 4, ... in groups of kHeadRows whose h rows are loaded together
  // (row by row, each row's load latency was exposed: 0.197 vs 0.143 ms for the three kernels)
  constexpr int kHeadRows = 4;
  for (int m0 = b0 + wv; m0 < b1; m0 += 4 * kHeadRows) {
    float hv[kHeadRows][kHeadCols], pre_r[kHeadRows], pre2_r[kHeadRows], tg_r[kHeadRows], rs_r[kHeadRows];
#pragma unroll
    for (int r = 0; r < kHeadRows; ++r) {
      const int m = m0 + 4 * r;
      const bool ok = m < b1;
#pragma unroll
      for (int q = 0; q < kHeadCols; ++q) {
        const int n = lane + 64 * q;
        hv[r][q] = (ok && n < N) ? h[(int64_t)m * ldh + n] : 0.f;
      }
      // the row's scalars with its h (loaded after the logit's reduction, each cost a full latency)
      pre_r[r] = (ok && oa.pre) ? oa.pre[m] : 0.f;
      pre2_r[r] = (ok && oa.pre2) ? oa.pre2[m] : 0.f;
      tg_r[r] = ok ? targets[m] : 0.f;
      rs_r[r] = 0.f;  // xDeepFM: the CIN's per-row partials, in tower_head_kernel's order
      if (ok && oa.rowsum)
        for (int j = 0; j < oa.rowsum_k; ++j) rs_r[r] += oa.rowsum[(int64_t)m * oa.rowsum_k + j];
    }
#pragma unroll
    for (int r = 0; r < kHeadRows; ++r) {
      const int m = m0 + 4 * r;
      if (m >= b1) break;
      float p = 0.f;
#pragma unroll
      for (int q = 0; q < kHeadCols; ++q)
        if (lane + 64 * q < N) p += hv[r][q] * wv4[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
      float y = p;
      if (oa.has_bo) y = y + oa.bo;
      if (oa.rowsum) y = rs_r[r] + y;
      if (oa.pre2) y = pre2_r[r] + y;
      float t = oa.pre ? pre_r[r] + y : y;
      t = t + oa.beta;
      const float x = 1.0f / (1.0f + expf(-t));
      const float tg = tg_r[r] > 0.f ? 1.f : 0.f;  // DeepFM.scala:106
      const float gp = -(tg - x) * norm / ((1.f - x + eps) * (x + eps));
      const float gz = gp * (1.f - x) * x;
      if (lane == 0) {
        oa.out[m] = x;
        dz[m] = gz;
      }
      if (lane == npend) {
        px = x;
        pt = tg;
        gsum += gz;
      }
      if (++npend == 64) flush();
#pragma unroll
      for (int q = 0; q < kHeadCols; ++q) {
        const int n = lane + 64 * q;
        if (n < N) {
          g[(int64_t)m * ldg + n] = hv[r][q] > 0.f ? gz * wv4[q] : 0.f;
          col[q] += gz * hv[r][q];
        }
      }
    }
  }
  flush();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    l += __shfl_xor(l, o);
    gsum += __shfl_xor(gsum, o);
  }
  if (lane == 0) {
    sl[wv] = l;
    sg[wv] = gsum;
  }
#pragma unroll
  for (int q = 0; q < kHeadCols; ++q) cs[wv][lane + 64 * q] = col[q];
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = ((sl[0] + sl[1]) + sl[2]) + sl[3];
    part[kMaxParts + blockIdx.x] = ((sg[0] + sg[1]) + sg[2]) + sg[3];
  }
  if (cpart)
    for (int n = threadIdx.x; n < N; n += 256)
      cpart[(int64_t)blockIdx.x * N + n] = ((cs[0][n] + cs[1][n]) + cs[2][n]) + cs[3][n];
}

// dPre of the last hidden layer: g[b][n] = dz[b] * wo[n] masked by ReLU (h > 0)
__global__ void head_back_kernel(int B, int N, const float* __restrict__ h, int ldh, const float* __restrict__ dz,
                                 const float* __restrict__ wo, float* __restrict__ g, int ldg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * N) return;
  const int64_t b = i / N;
  const int n = (int)(i - b * N);
  g[b * ldg + n] = h[b * ldh + n] > 0.f ? dz[b] * wo[n] : 0.f;
}

// the same, four columns per thread (16-B loads / stores; N, ldh, ldg multiples of 4)
__global__ void head_back4_kernel(int B, int N4, const float4* __restrict__ h, int ldh4, const float* __restrict__ dz,
                                  const float4* __restrict__ wo, float4* __restrict__ g, int ldg4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * N4) return;
  const int64_t b = i / N4;
  const int n = (int)(i - b * N4);
  const float4 hv = h[b * ldh4 + n], w = wo[n];
  const float d = dz[b];
  g[b * ldg4 + n] = make_float4(hv.x > 0.f ? d * w.x : 0.f, hv.y > 0.f ? d * w.y : 0.f, hv.z > 0.f ? d * w.z : 0.f,
                                hv.w > 0.f ? d * w.w : 0.f);
}

// BigDL ReLU backward (Threshold(0, 0)): g *= (h > 0), in place
__global__ void relu_back_kernel(int B, int N, const float* __restrict__ h, int ldh, float* __restrict__ g,
                                 int ldg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * N) return;
  const int64_t b = i / N;
  const int n = (int)(i - b * N);
  if (!(h[b * ldh + n] > 0.f)) g[b * ldg + n] = 0.f;
}

// dL/dE[b][f][j] = dx[b][f*k + j] (+ FM: dz[b] * (s_j - e[b][f][j]) / k), thread per (b, j)
__global__ void emb_grad_kernel(int B, int F, int k, const float* __restrict__ x, int ldx,
                                const float* __restrict__ dx, int lddx, const float* __restrict__ dz, int fm,
                                const float* __restrict__ gx0, float* __restrict__ gE) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * k) return;
  const int64_t b = i / k;
  const int j = (int)(i - b * k);
  const float* xr = x + b * ldx;
  float s = 0.f;
  if (fm)
    for (int f = 0; f < F; ++f) s += xr[f * k + j];
  const float gz = fm ? dz[b] : 0.f;
  for (int f = 0; f < F; ++f) {
    float v = dx ? dx[b * lddx + f * k + j] : 0.f;
    if (fm) v += gz * (s - xr[f * k + j]) / (float)k;
    if (gx0) v += gx0[(b * k + j) * F + f];  // xDeepFM: CIN part (x0[b*k + j][f] = e[b][f][j])
    gE[(b * F + f) * k + j] = v;
  }
}

// Scatter backward: dL/dw[n] = dz[index[n]] (index null: n / F)
__global__ void w_grad_kernel(int64_t nnz, int F, const int32_t* __restrict__ index, const float* __restrict__ dz,
                              float* __restrict__ gw) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= nnz) return;
  gw[n] = dz[index ? index[n] : (int)(n / F)];
}

// DCN cross stack backward, per row, in the closed form x_l = a_l x0 + c_l 1 (a_0 = 1, c_0 = 0,
// s_l = w_l . x_l = a_l u_l + c_l sum(w_l), a_{l+1} = a_l + s_l, c_{l+1} = c_l + beta_l;
// y = a_L v + c_L sum(W_out[0:D])).  With g = dL/dz, going down the stack the gradient of x_l is
// g W_out + sum_{m >= l} gs_m w_m, where gs_l = g v + sum_{m > l} gs_m u_m (scalar).  Hence
//   dL/dx0   = g a_L W_out + sum_m gs_m a_m w_m                 -> coef[b] = [gs_0 a_0 .. | g a_L]
//   dL/dw_m  = sum_b gs_m (a_m x0 + c_m)                         -> coef^T x0 + cst sums
//   dL/dW_out[0:D] = sum_b g (a_L x0 + c_L)
//   dL/dbeta_l = sum_b (g sum(W_out) + sum_{m > l} gs_m sum(w_m))
// cst[b] = [gs_0 c_0 .. gs_{L-1} c_{L-1}, g c_L, gb_0 .. gb_{L-1}]  (summed over b by a GEMV).
__global__ void cross_back_kernel(int B, int L, const float* __restrict__ xcol, CrossScalars cs,
                                  const float* __restrict__ dz, float* __restrict__ coef, float* __restrict__ cst) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* u = xcol + (int64_t)b * (L + 1);
  float a[kMaxFusedCross + 1], c[kMaxFusedCross + 1];
  a[0] = 1.f;
  c[0] = 0.f;
  for (int l = 0; l < L; ++l) {
    const float sl = a[l] * u[l] + c[l] * cs.wsum[l];
    a[l + 1] = a[l] + sl;
    c[l + 1] = c[l] + cs.beta[l];
  }
  const float g = dz[b];
  float* cf = coef + (int64_t)b * (L + 1);
  float* ct = cst + (int64_t)b * (2 * L + 1);
  cf[L] = g * a[L];
  ct[L] = g * c[L];
  float run = g * u[L];              // g v + sum_{m > l} gs_m u_m
  float gbr = g * cs.wo_sum;         // g sum(W_out) + sum_{m > l} gs_m sum(w_m)
  for (int l = L - 1; l >= 0; --l) {
    const float gs = run;
    ct[L + 1 + l] = gbr;
    cf[l] = gs * a[l];
    ct[l] = gs * c[l];
    run += gs * u[l];
    gbr += gs * cs.wsum[l];
  }
}

// gwc[r][d] + colsum[r] -> the mats slots: rows < L at w_off + r*D, row L at wo_off
__global__ void cross_wgrad_kernel(int L, int D, const float* __restrict__ gwc, const float* __restrict__ csum,
                                   float* __restrict__ gw, float* __restrict__ gwo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (L + 1) * D) return;
  const int r = i / D, d = i - r * D;
  const float v = gwc[i] + csum[r];
  if (r < L) gw[(int64_t)r * D + d] = v;
  else gwo[d] = v;
}

__global__ void copy_kernel(int n, const float* __restrict__ x, float* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i];
}

// y[0] = sum_i x[i] (one thread, fixed order)
__global__ void sum_kernel(int n, const float* __restrict__ x, float* __restrict__ y) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += x[i];
  *y = (float)s;
}

// PNN: dL/dE[b][f][j] = dx[b][f*k + j] + sum_{g != f} dip[b][pair(f, g)] * e[b][g][j]
// (DotProduct2 backward, ProductEncoder.scala:43-70), pairs (i < j) lexicographic.
__global__ void pnn_emb_grad_kernel(int B, int F, int k, const float* __restrict__ x, int ldx,
                                    const float* __restrict__ dx, int lddx, float* __restrict__ gE) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * F * k) return;
  const int64_t b = i / (F * k);
  const int r = (int)(i - b * F * k), f = r / k, j = r - f * k;
  const float* xr = x + b * ldx;
  const float* dip = dx + b * lddx + F * k;
  float v = dx[b * lddx + r];
  for (int g = 0; g < F; ++g) {
    if (g == f) continue;
    const int lo = f < g ? f : g, hi = f < g ? g : f;
    const int p = lo * (2 * F - lo - 1) / 2 + (hi - lo - 1);
    v += dip[p] * xr[g * k + j];
  }
  gE[i] = v;
}

// ---- xDeepFM CIN backward (CINEncoder.scala:60-103; forward semantics in k_gemm.hip) ----
__global__ void cin_x0_kernel(int B, int F, int k, const float* __restrict__ x, int ldx, float* __restrict__ x0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * k * F) return;
  const int64_t r = i / F;
  const int f = (int)(i - r * F);
  const int64_t b = r / k;
  const int j = (int)(r - b * k);
  x0[i] = x[b * ldx + f * k + j];
}

__global__ void expand_dz_kernel(int64_t R, int k, const float* __restrict__ dz, float* __restrict__ dzr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) dzr[r] = dz[r / k];
}

// gpre[r][h] = ReLU'(u_l) * (gu[r][h] (from layer l+1) + dz[b] * W_out[slice_l + h] (pooling: Sum over k))
__global__ void cin_gpre_kernel(int64_t R, int H, int k, const float* __restrict__ u, int ldu,
                                const float* __restrict__ gu, const float* __restrict__ dz,
                                const float* __restrict__ wo, float* __restrict__ gpre) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * H) return;
  const int64_t r = i / H;
  const int h = (int)(i - r * H);
  float g = dz[r / k] * wo[h];
  if (gu) g += gu[r * ldu + h];
  gpre[r * ldu + h] = u[r * ldu + h] > 0.f ? g : 0.f;
}

// z[r][f*Hp + h] = x0[r][f] * up[r][h]  (MM(transB) of (F x 1)(1 x Hp), CINEncoder.scala:152)
__global__ void cin_z_kernel(int64_t rows, int F, int Hp, const float* __restrict__ x0,
                             const float* __restrict__ up, int ldu, float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int FH = F * Hp;
  if (i >= rows * FH) return;
  const int64_t r = i / FH;
  const int c = (int)(i - r * FH), f = c / Hp, h = c - f * Hp;
  z[i] = x0[r * F + f] * up[r * ldu + h];
}

// gx0[r][f] += sum_h gz[r][f*Hp + h] * up[r][h]: one block per row, wave w takes f = w, w + 4, ...,
// lanes stride h (coalesced 256-B reads of gz), shuffle reduction per f (fixed order).
__global__ __launch_bounds__(256) void cin_back_x0_kernel(int64_t rows, int F, int Hp, const float* __restrict__ gz,
                                                          int ldz, const float* __restrict__ up, int ldu,
                                                          float* __restrict__ gx0) {
  const int64_t r = blockIdx.x;
  if (r >= rows) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* uu = up + r * ldu;
  const float* g = gz + r * (int64_t)ldz;
  for (int f = w; f < F; f += 4) {
    float acc = 0.f;
    for (int h = lane; h < Hp; h += 64) acc += g[(int64_t)f * Hp + h] * uu[h];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) gx0[r * F + f] += acc;
  }
}

// out[r][h] (=, or += when accum) sum_f gz[r][f*Hp + h] * x0[r][f]
__global__ void cin_back_u_kernel(int64_t rows, int F, int Hp, const float* __restrict__ gz, int ldz,
                                  const float* __restrict__ x0, float* __restrict__ out, int ldo, int accum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * Hp) return;
  const int64_t r = i / Hp;
  const int h = (int)(i - r * Hp);
  const float* g = gz + r * (int64_t)ldz + h;
  const float* xr = x0 + r * F;
  float acc = 0.f;
  for (int f = 0; f < F; ++f) acc += g[(int64_t)f * Hp] * xr[f];
  if (accum) out[r * ldo + h] += acc;
  else out[r * ldo + h] = acc;
}

// Both contractions of dL/dz in one pass over it (one block per row r; the two kernels above read
// the 4 x F x Hp bytes of each row twice):
//   gx0[r][f] += sum_h gz[r][f*Hp + h] * up[r][h]   (f-row partials of VEC columns per thread,
//                                                     then summed over the row in h order)
//   out[r][h] (=, or += when accum) sum_f gz[r][f*Hp + h] * x0[r][f]   (G interleaved f-groups,
//                                                     each in ascending f, then the groups in order)
// Thread t owns columns [VEC hw, VEC hw + VEC) (hw = t % HW, HW = Hp / VEC) of f-group fg = t / HW.
// gx0 is updated before out (layer 0: both are the x0 gradient).  Fixed orders: deterministic.
template <int VEC>
__global__ __launch_bounds__(256) void cin_back_fused_kernel(int64_t rows, int F, int Hp, const float* __restrict__ gz,
                                                             int ldz, const float* __restrict__ up, int ldup,
                                                             const float* __restrict__ x0, float* gx0, float* out,
                                                             int ldo, int accum) {
  extern __shared__ float cbf_sm[];
  const int64_t r = blockIdx.x;
  if (r >= rows) return;
  const int HW = Hp / VEC, G = 256 / HW;
  const int t = threadIdx.x, hw = t % HW, fg = t / HW;
  float* redx = cbf_sm;           // [F][HW]
  float* redu = cbf_sm + F * HW;  // [G][Hp]
  if (fg < G) {
    float uv[VEC], gacc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      uv[e] = up[r * ldup + hw * VEC + e];
      gacc[e] = 0.f;
    }
    const float* g = gz + r * (int64_t)ldz + hw * VEC;
    for (int f = fg; f < F; f += G) {
      float v[VEC];
      if constexpr (VEC == 4) {
        const float4 q = *reinterpret_cast<const float4*>(g + (int64_t)f * Hp);
        v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
      } else {
        v[0] = g[(int64_t)f * Hp];
      }
      const float xf = x0[r * F + f];
      float pd = 0.f;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        gacc[e] += v[e] * xf;
        pd += v[e] * uv[e];
      }
      redx[f * HW + hw] = pd;
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) redu[fg * Hp + hw * VEC + e] = gacc[e];
  }
  __syncthreads();
  for (int f = t; f < F; f += 256) {  // every field, also F > 256
    float sx = 0.f;
    for (int i = 0; i < HW; ++i) sx += redx[f * HW + i];
    gx0[r * F + f] += sx;
  }
  __syncthreads();
  for (int h = t; h < Hp; h += 256) {
    float su = 0.f;
    for (int q = 0; q < G; ++q) su += redu[q * Hp + h];
    if (accum) out[r * ldo + h] += su;
    else out[r * ldo + h] = su;
  }
}

// ---- small / irregular fp32 GEMMs of the backward (replaces the library sgemm) ----
// C[m][n] (= or += when ACC) sum_k A[m][k] * B(k, n), B(k, n) = B[k * ldb + n] (row-major K x N) or,
// with BT, B[n * ldb + k] (row-major N x K).  64 x 64 block tiles, 4 waves of 32 x 32 (2 x 2 tiles of
// v_mfma_f32_16x16x4_f32: an exact fp32 FMA chain), K in 16-wide LDS chunks, zero-filled edges.
// Used for the tower dX of layers without split-GEMM W^T planes and the DCN cross GEMMs (K or N of
// the cross width L + 1).
template <bool BT, bool ACC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                      const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                      int ldc) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float As[64][17];  // [row][k]
  __shared__ float Bs[16][65];  // [k][col]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int wr = (wid >> 1) * 32, wc = (wid & 1) * 32;
  const int g = lane >> 4, r16 = lane & 15;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // A: 64 x 16, consecutive threads along k
      const int e = tid + q * 256, r = e >> 4, c = e & 15;
      const int m = m0 + r, k = k0 + c;
      As[r][c] = (m < M && k < K) ? A[(int64_t)m * lda + k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // B: 16 x 64
      const int e = tid + q * 256;
      int kk, nn;
      if (BT) {
        nn = e >> 4;
        kk = e & 15;
      } else {
        kk = e >> 6;
        nn = e & 63;
      }
      const int k = k0 + kk, n = n0 + nn;
      Bs[kk][nn] = (k < K && n < N) ? (BT ? B[(int64_t)n * ldb + k] : B[(int64_t)k * ldb + n]) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int kk = s4 * 4 + g;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float a = As[wr + i * 16 + r16][kk];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[kk][wc + j * 16 + r16], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr + i * 16 + g * 4 + r, n = n0 + wc + j * 16 + r16;
        if (m < M && n < N) {
          float* c = C + (int64_t)m * ldc + n;
          *c = ACC ? *c + acc[i][j][r] : acc[i][j][r];
        }
      }
}

int launch_gemm_f32(hipStream_t s, bool bt, bool accumulate, int M, int N, int K, const float* A, int lda,
                    const float* B, int ldb, float* C, int ldc) {
  if (M <= 0 || N <= 0) return RMX_OK;
  dim3 grid((M + 63) / 64, (N + 63) / 64);
#define RMX_G(bt_, acc_) hipLaunchKernelGGL((gemm_f32_kernel<bt_, acc_>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc)
  if (bt) {
    if (accumulate) RMX_G(true, true);
    else RMX_G(true, false);
  } else {
    if (accumulate) RMX_G(false, true);
    else RMX_G(false, false);
  }
#undef RMX_G
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// ---- weight gradients: dW[n][k] = sum_r A[r][n] X[r][k] (reduction over the batch rows) ----
// The "TN" GEMM of every Linear backward.  Both operands are row-major over the reduction index,
// so a block stages 16-row chunks of A[:, n0:n0+64] and X[:, k0:k0+64] TRANSPOSED into LDS tile
// images [col][16 rows] (one 64-B row per column; the row quartets of lane group g are 16-B slots,
// XOR-swizzled as the forward engine's, k_gemm.hpp) with one ds_write_b128 per thread, and reads
// MFMA fragments with ds_read_b128: lane (i = l & 15, g = l >> 4) holds rows 4g..4g+3 of column i,
// feeding 4 k-steps of v_mfma_f32_16x16x4_f32.  4 waves in 2 x 2, 32 x 32 outputs each.  The rows
// are split into S slices (grid.y) for parallelism; each block writes its partial tile to
// part[slice][N][K] and wgrad_reduce_kernel sums the slices in fixed order (deterministic).
constexpr int kWgT = 64;  // block tile (n and k)

__device__ __forceinline__ int wg_slot(int col, int g) { return g ^ ((4 - ((col >> 2) & 3)) & 3); }

__global__ __launch_bounds__(256) void wgrad_kernel(int rows, int N, int K, const float* __restrict__ A, int lda,
                                                    const float* __restrict__ X, int ldx, int rows_per_slice,
                                                    int tiles, float* __restrict__ part) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float lds[2][2][kWgT * 16];  // [buf][A|X][col][16]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // XCD-aware order: consecutive block ids go to the 8 XCDs round robin, so XCD x runs slices
  // x, x + 8, ... and all tiles of a slice share its L2 (the slice's rows are fetched once per XCD)
  const int bid = blockIdx.x, xcd = bid & 7, idx = bid >> 3;
  const int slice = (idx / tiles) * 8 + xcd, tile = idx % tiles;
  const int ntn = (N + kWgT - 1) / kWgT;
  const int n0 = (tile % ntn) * kWgT, k0 = (tile / ntn) * kWgT;
  const int r_begin = slice * rows_per_slice;
  const int r_end = min(rows, r_begin + rows_per_slice);
  const int nch = r_end > r_begin ? (r_end - r_begin + 15) / 16 : 0;
  // staging item: column = lane, row quartet h = wid (rows 4h..4h+3 of the chunk)
  const int col = lane, h = wid;
  float4 ra, rx;
  auto gload = [&](int c) {
    const int r0 = r_begin + c * 16 + 4 * h;
    float va[4], vx[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + q;
      const bool ok = r < r_end;
      va[q] = (ok && n0 + col < N) ? A[(int64_t)r * lda + n0 + col] : 0.f;
      vx[q] = (ok && k0 + col < K) ? X[(int64_t)r * ldx + k0 + col] : 0.f;
    }
    ra = make_float4(va[0], va[1], va[2], va[3]);
    rx = make_float4(vx[0], vx[1], vx[2], vx[3]);
  };
  auto sstore = [&](int buf) {
    const int off = col * 16 + wg_slot(col, h) * 4;
    *reinterpret_cast<float4*>(&lds[buf][0][off]) = ra;
    *reinterpret_cast<float4*>(&lds[buf][1][off]) = rx;
  };
  const int wi = wid >> 1, wj = wid & 1, g = lane >> 4, r16 = lane & 15;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nch > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) gload(c + 1);
    f32x4 fa[2], fx[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ca = wi * 32 + t * 16 + r16, cx = wj * 32 + t * 16 + r16;
      fa[t] = *reinterpret_cast<const f32x4*>(&lds[cur][0][ca * 16 + wg_slot(ca, g) * 4]);
      fx[t] = *reinterpret_cast<const f32x4*>(&lds[cur][1][cx * 16 + wg_slot(cx, g) * 4]);
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a][s4], fx[b][s4], acc[a][b], 0, 0, 0);
    if (c + 1 < nch) sstore(cur ^ 1);
    __syncthreads();
  }
  float* out = part + (int64_t)slice * N * K;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int k = k0 + wj * 32 + b * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wi * 32 + a * 16 + 4 * g + r;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[a][b][r];
      }
    }
}

// The same "TN" GEMM on the bf16 matrix cores through the exact 3-way split (k_gemm.hpp kPrecS3,
// DESIGN.md §4): both operands are fp32 activations / gradients, so they are split while staged --
// each element once per block -- into three bf16 planes of LDS images [col][32 rows] (64-B rows,
// 16-B slots of 8 rows XOR-swizzled by wg_slot); a wave's fragment of a 16-column tile is one
// ds_read_b128 per plane, and a 32-row chunk costs 6 v_mfma_f32_16x16x32_bf16 per output tile
// (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid, smallest first) against 8 f32 MFMAs per 16 rows.
typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kWgR = 32;  // rows per chunk (the MFMA K)
// timing-only diagnostic builds (tools/diag_build.sh-style, results wrong): 1 = no LDS stores in the
// loop, 2 = no MFMAs, 4 = no global loads in the loop
#ifndef RMX_WGRAD_DIAG
#define RMX_WGRAD_DIAG 0
#endif

__device__ __forceinline__ void wg_split(const float* v, wg_bf16x8& hi, wg_bf16x8& mi, wg_bf16x8& lo) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const __bf16 h = (__bf16)v[q];
    const float r = v[q] - (float)h;
    const __bf16 m = (__bf16)r;
    hi[q] = h;
    mi[q] = m;
    lo[q] = (__bf16)(r - (float)m);
  }
}

// GZ: the X operand is the CIN outer product z[r][f * Hp + h] = x0[r][f] * up[r][h] (CINEncoder.scala:152),
// generated while staged (the same fp32 product cin_z_kernel stores) instead of read from memory
struct WgZ {
  const float* x0 = nullptr;  // [rows][F]
  const float* up = nullptr;  // [rows][ldup]
  int F = 0, Hp = 0, ldup = 0;
};

// TT x TT output tile per block (TT = 64: 2 x 2 waves of 32 x 32; TT = 128: 2 x 4 waves of 64 x 32,
// halving the L2 reads and LDS fragment reads per output), LDS [buf][A | X][plane][col][32 rows] bf16.
// SB (knob "wgrad_sb"): one LDS buffer (48 KiB at TT = 128) and a second barrier per chunk, so two
// blocks share a CU (4 waves per SIMD): one block's MFMAs run while the other splits and stores its
// next chunk, where the double-buffered block's waves all reach that phase together.  Same chunks,
// same MFMA order per output: bitwise the same gradients.
template <int TT, bool GZ = false, bool SB = false>
__global__ __launch_bounds__(TT == 64 ? 256 : 512, SB ? 4 : 1) void wgrad_s3_kernel(int rows, int N, int K,
                                                                        const float* __restrict__ A, int lda,
                                                                        const float* __restrict__ X, int ldx,
                                                                        int rows_per_slice, int tiles,
                                                                        float* __restrict__ part, WgZ zg) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int WJ = TT == 64 ? 2 : 4, TI = TT == 64 ? 2 : 4, TJ = 2;  // waves along k; tiles per wave
  extern __shared__ __attribute__((aligned(16))) wg_bf16x8 wlds[];
  auto L = [&](int buf, int op, int pl) { return wlds + ((buf * 2 + op) * 3 + pl) * TT * 4; };
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, xcd = bid & 7, idx = bid >> 3;
  const int slice = (idx / tiles) * 8 + xcd, tile = idx % tiles;
  const int ntn = (N + TT - 1) / TT;
  const int n0 = (tile % ntn) * TT, k0 = (tile / ntn) * TT;
  const int r_begin = slice * rows_per_slice;
  const int r_end = min(rows, r_begin + rows_per_slice);
  const int nch = r_end > r_begin ? (r_end - r_begin + kWgR - 1) / kWgR : 0;
  // staging item: column tid % TT, row octet h = tid / TT (rows 8h..8h+7 of the chunk)
  const int col = tid % TT, h = tid / TT;
  const bool a_ok = n0 + col < N, x_ok = k0 + col < K;
  const int zf = GZ ? (k0 + col) / zg.Hp : 0, zh = GZ ? k0 + col - zf * zg.Hp : 0;  // (f, h) of column k
  // two register sets: the loads of chunk c + 2 are in flight while chunk c computes and chunk c + 1
  // (loaded two steps earlier) is split into LDS
  float a0[8], x0[8], a1[8], x1[8];
  auto gload = [&](int c, float* va, float* vx) {
    const int r0 = r_begin + c * kWgR + 8 * h;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = r0 + q;
      const bool ok = r < r_end;
      va[q] = (ok && a_ok) ? A[(int64_t)r * lda + n0 + col] : 0.f;
      if constexpr (GZ)
        vx[q] = (ok && x_ok) ? zg.x0[(int64_t)r * zg.F + zf] * zg.up[(int64_t)r * zg.ldup + zh] : 0.f;
      else
        vx[q] = (ok && x_ok) ? X[(int64_t)r * ldx + k0 + col] : 0.f;
    }
  };
  auto sstore = [&](int buf, const float* va, const float* vx) {
    const int o = col * 4 + wg_slot(col, h);
    wg_bf16x8 p0, p1, p2;
    wg_split(va, p0, p1, p2);
    L(buf, 0, 0)[o] = p0;
    L(buf, 0, 1)[o] = p1;
    L(buf, 0, 2)[o] = p2;
    wg_split(vx, p0, p1, p2);
    L(buf, 1, 0)[o] = p0;
    L(buf, 1, 1)[o] = p1;
    L(buf, 1, 2)[o] = p2;
  };
  const int wi = wid / WJ, wj = wid - (wid / WJ) * WJ, g = lane >> 4, r16 = lane & 15;
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int cur) {
    if constexpr (RMX_WGRAD_DIAG & 2) return;
    // SB: an A fragment is read just before its MFMAs (fewer live VGPRs for 4 waves per SIMD)
    wg_bf16x8 fa[SB ? 1 : TI][3], fx[TJ][3];
    auto lda_frag = [&](int t, wg_bf16x8* f) {
      const int ca = wi * TI * 16 + t * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) f[pl] = L(cur, 0, pl)[ca * 4 + wg_slot(ca, g)];
    };
    if constexpr (!SB)
#pragma unroll
      for (int t = 0; t < TI; ++t) lda_frag(t, fa[t]);
#pragma unroll
    for (int t = 0; t < TJ; ++t) {
      const int cx = wj * TJ * 16 + t * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fx[t][pl] = L(cur, 1, pl)[cx * 4 + wg_slot(cx, g)];
    }
#pragma unroll
    for (int ai = 0; ai < TI; ++ai) {
      if constexpr (SB) lda_frag(ai, fa[0]);
      const int a = SB ? 0 : ai;
#pragma unroll
      for (int b = 0; b < TJ; ++b) {
        f32x4 d = acc[ai][b];
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][1], fx[b][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][2], fx[b][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][0], fx[b][2], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][1], fx[b][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][0], fx[b][1], d, 0, 0, 0);
        acc[ai][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a][0], fx[b][0], d, 0, 0, 0);
      }
    }
  };
  if (nch > 0) {
    gload(0, a0, x0);
    sstore(0, a0, x0);
  }
  if (nch > 1) gload(1, a0, x0);
  if (!SB && nch > 2) gload(2, a1, x1);
  __syncthreads();
  if constexpr (SB) {
    // one register set (no spills at 4 waves per SIMD): chunk c + 2's loads fly during chunk c + 1's
    // MFMAs; the partner block's MFMAs cover this block's split / store phase
    for (int c = 0; c < nch; ++c) {
      compute(0);
      __syncthreads();  // every wave is done reading the one buffer
      if (c + 1 < nch) {
        if (!(RMX_WGRAD_DIAG & 1)) sstore(0, a0, x0);
        if (!(RMX_WGRAD_DIAG & 4) && c + 2 < nch) gload(c + 2, a0, x0);
      }
      __syncthreads();
    }
  }
  constexpr int B1 = 1;  // the odd chunks' buffer
  for (int c = 0; !SB && c < nch; c += 2) {
    compute(0);  // chunk c (even) in buffer 0
    if (c + 1 < nch) {
      if (!(RMX_WGRAD_DIAG & 1)) sstore(B1, a0, x0);
      if (!(RMX_WGRAD_DIAG & 4) && c + 3 < nch) gload(c + 3, a0, x0);
    }
    __syncthreads();
    if (c + 1 >= nch) break;
    compute(B1);  // chunk c + 1
    if (c + 2 < nch) {
      if (!(RMX_WGRAD_DIAG & 1)) sstore(0, a1, x1);
      if (!(RMX_WGRAD_DIAG & 4) && c + 4 < nch) gload(c + 4, a1, x1);
    }
    __syncthreads();
  }
  float* out = part + (int64_t)slice * N * K;
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) {
      const int k = k0 + wj * TJ * 16 + b * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wi * TI * 16 + a * 16 + 4 * g + r;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[a][b][r];
      }
    }
}

// The same single-buffered split dW on a 208 x 128 tile (knob "wgrad_nk", default on for the CIN): n (the dPre /
// gpre columns) in 13 MFMA tiles, so N = 400 pads to 416 and the CIN's N = 200 to 208 instead of 512 /
// 256 on the square 128 tiles (19-28 % fewer MFMAs, fewer blocks); k in 128.  8 waves, wave w owns
// k tile w and all 13 n tiles.  Staging items (col, row octet): [208 A cols | 128 X cols] x 4 octets,
// up to 3 per thread.  Per output the chunks and the 6 MFMAs run in the same order as the 128 x 128
// kernel; only the row-slice split S (a function of the tile count) can differ.
constexpr int kNkN = 208, kNkK = 128, kNkItems = (kNkN + kNkK) * 4, kNkPer = (kNkItems + 511) / 512;
template <bool GZ>
__global__ __launch_bounds__(512, 4) void wgrad_nk_kernel(int rows, int N, int K, const float* __restrict__ A, int lda,
                                                          const float* __restrict__ X, int ldx, int rows_per_slice,
                                                          int tiles, float* __restrict__ part, WgZ zg) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) wg_bf16x8 wlds[];
  // LDS [A planes 3][208 cols][4 slots] then [X planes 3][128 cols][4 slots]
  auto LA = [&](int pl) { return wlds + pl * kNkN * 4; };
  auto LX = [&](int pl) { return wlds + 3 * kNkN * 4 + pl * kNkK * 4; };
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, xcd = bid & 7, idx = bid >> 3;
  const int slice = (idx / tiles) * 8 + xcd, tile = idx % tiles;
  const int ntn = (N + kNkN - 1) / kNkN;
  const int n0 = (tile % ntn) * kNkN, k0 = (tile / ntn) * kNkK;
  const int r_begin = slice * rows_per_slice;
  const int r_end = min(rows, r_begin + rows_per_slice);
  const int nch = r_end > r_begin ? (r_end - r_begin + kWgR - 1) / kWgR : 0;
  // this thread's staging items, packed col | h << 8 | op << 10 | ok << 11 (few live VGPRs), and (GZ)
  // the (f, h) of an X column
  int it[kNkPer], it_zf[kNkPer], it_zh[kNkPer];
#pragma unroll
  for (int q = 0; q < kNkPer; ++q) {
    const int i = tid + q * 512;
    const bool a = i < kNkN * 4;
    const int j = a ? i : i - kNkN * 4;
    const int col = a ? j % kNkN : j % kNkK, h = a ? j / kNkN : j / kNkK;
    const bool ok = i < kNkItems && (a ? n0 + col < N : k0 + col < K);
    it[q] = col | h << 8 | (a ? 0 : 1) << 10 | (ok ? 1 : 0) << 11;
    const int kk = k0 + col;
    it_zf[q] = GZ && !a ? kk / zg.Hp : 0;
    it_zh[q] = GZ && !a ? kk - it_zf[q] * zg.Hp : 0;
  }
  float v[kNkPer][8];
  auto gload = [&](int c) {
#pragma unroll
    for (int q = 0; q < kNkPer; ++q) {
      const int col = it[q] & 255, h = (it[q] >> 8) & 3, op = (it[q] >> 10) & 1;
      const bool ok = (it[q] >> 11) & 1;
      const int r0 = r_begin + c * kWgR + 8 * h;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int r = r0 + e;
        float x = 0.f;
        if (ok && r < r_end) {
          if (op == 0)
            x = A[(int64_t)r * lda + n0 + col];
          else if constexpr (GZ)
            x = zg.x0[(int64_t)r * zg.F + it_zf[q]] * zg.up[(int64_t)r * zg.ldup + it_zh[q]];
          else
            x = X[(int64_t)r * ldx + k0 + col];
        }
        v[q][e] = x;
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int q = 0; q < kNkPer; ++q) {
      if (tid + q * 512 >= kNkItems) continue;
      const int col = it[q] & 255, o = col * 4 + wg_slot(col, (it[q] >> 8) & 3);
      wg_bf16x8 p0, p1, p2;
      wg_split(v[q], p0, p1, p2);
      if (((it[q] >> 10) & 1) == 0) {
        LA(0)[o] = p0;
        LA(1)[o] = p1;
        LA(2)[o] = p2;
      } else {
        LX(0)[o] = p0;
        LX(1)[o] = p1;
        LX(2)[o] = p2;
      }
    }
  };
  const int g = lane >> 4, r16 = lane & 15;
  f32x4 acc[13];
#pragma unroll
  for (int a = 0; a < 13; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&]() {
    wg_bf16x8 fx[3], fa[3];
    const int cx = wid * 16 + r16;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) fx[pl] = LX(pl)[cx * 4 + wg_slot(cx, g)];
#pragma unroll
    for (int a = 0; a < 13; ++a) {
      const int ca = a * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fa[pl] = LA(pl)[ca * 4 + wg_slot(ca, g)];
      f32x4 d = acc[a];
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[2], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[1], d, 0, 0, 0);
      acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[0], d, 0, 0, 0);
    }
  };
  if (nch > 0) {
    gload(0);
    sstore();
  }
  if (nch > 1) gload(1);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    compute();
    __syncthreads();  // every wave is done reading the one buffer
    if (c + 1 < nch) {
      sstore();
      if (c + 2 < nch) gload(c + 2);
    }
    __syncthreads();
  }
  float* out = part + (int64_t)slice * N * K;
  const int k = k0 + wid * 16 + r16;
#pragma unroll
  for (int a = 0; a < 13; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + a * 16 + 4 * g + r;
      if (n < N && k < K) out[(int64_t)n * K + k] = acc[a][r];
    }
}

// The split dW on a 208 x 208 tile (knob "wgrad_sq", the tower's dW = dPre^T x_in): 13 waves, wave w owns
// k tile w and all 13 n tiles (13 x 6 MFMAs per 32-row chunk), one block per CU on a double-buffered
// 156 KiB LDS image.  Against the 128 x 128 tiles, a 400 x 400 dW is 2 x 2 tiles instead of 4 x 4 (416^2
// instead of 512^2 outputs computed) and every batch row is staged 2 + 2 times instead of 4 + 4 -- the
// staging (loads, split, LDS stores), not the MFMAs, is what the dW waits on.  Each
// thread stages one A and one X item (a column's 8-row octet) per chunk; the loads of chunk c + 2 fly
// during chunk c + 1's MFMAs, and chunk c + 1 is split and stored into the other buffer while chunk c
// computes.  Per output the chunks and the 6 MFMAs run in the same order as the 128 x 128 kernel; only
// the row-slice split S can differ.
constexpr int kSqT = 208, kSqW = kSqT / 16, kSqThr = kSqW * 64;
// cpart (nullable): the blocks of the first k tile also sum their A columns over their row slice (the
// bias gradient, sum_b dPre[b][n], fused: the A items pass through registers anyway) into
// cpart[slice][N], rows in order per staging thread, the 4 row octets added in order at the end.
// GZ: X is the CIN outer product z = x0 (x) up generated while staged (as wgrad_s3_kernel / wgrad_nk_kernel).
// DG (timing probes, results wrong; knob "wgrad_diag"): 1 no MFMAs, 2 no staging (loads, split, LDS
// stores), 4 no LDS fragment reads.
// W16 (knob "wgrad_sq16"): 16 waves instead of 13, so each SIMD carries 4 waves of nearly equal MFMA work: with
// 13, SIMD 0 holds waves 0, 4, 8, 12 (4 x 13 tiles) against 3 x 13 on the others, and the block waits for it.
// Waves 0 .. 12 keep their k tile and take n tiles 0 .. 9; waves 13, 14, 15 take n tile 10, 11, 12 across all
// 13 k tiles (per SIMD 40 / 43 / 43 / 43 tiles).  Each output still sees the same chunks and products in the
// same order: bitwise the 13-wave kernel.  Threads past the 832 staging items only compute.
constexpr int kSq16Thr = 1024;
template <bool GZ, int DG = 0, bool W16 = false>
__global__ __launch_bounds__(W16 ? kSq16Thr : kSqThr, 1) void wgrad_sq_kernel(int rows, int N, int K, const float* __restrict__ A,
                                                             int lda, const float* __restrict__ X, int ldx,
                                                             int rows_per_slice, int tiles, float* __restrict__ part,
                                                             float* __restrict__ cpart, WgZ zg) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) wg_bf16x8 wlds[];
  // [buf][op: A, X][plane][208 cols][4 slots]
  auto L = [&](int buf, int op, int pl) { return wlds + ((buf * 2 + op) * 3 + pl) * kSqT * 4; };
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, xcd = bid & 7, idx = bid >> 3;
  const int slice = (idx / tiles) * 8 + xcd, tile = idx % tiles;
  const int ntn = (N + kSqT - 1) / kSqT;
  const int n0 = (tile % ntn) * kSqT, k0 = (tile / ntn) * kSqT;
  const int r_begin = slice * rows_per_slice;
  const int r_end = min(rows, r_begin + rows_per_slice);
  const int nch = r_end > r_begin ? (r_end - r_begin + kWgR - 1) / kWgR : 0;
  // staging item of this thread: column col of A (n0 + col) and of X (k0 + col), row octet h
  const int col = tid % kSqT, h = tid / kSqT;
  const bool stager = !W16 || tid < kSqThr;  // (W16: threads 832 .. 1023 stage nothing)
  const bool a_ok = stager && n0 + col < N, x_ok = stager && k0 + col < K;
  const bool csum_on = cpart != nullptr && k0 == 0;
  const int zf = GZ ? (k0 + col) / zg.Hp : 0, zh = GZ ? k0 + col - zf * zg.Hp : 0;  // (f, h) of column k
  float va[8], vx[8], csum = 0.f;
  auto gload = [&](int c) {
    const int r0 = r_begin + c * kWgR + 8 * h;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = r0 + q;
      const bool ok = r < r_end;
      va[q] = (ok && a_ok) ? A[(int64_t)r * lda + n0 + col] : 0.f;
      if constexpr (GZ)
        vx[q] = (ok && x_ok) ? zg.x0[(int64_t)r * zg.F + zf] * zg.up[(int64_t)r * zg.ldup + zh] : 0.f;
      else
        vx[q] = (ok && x_ok) ? X[(int64_t)r * ldx + k0 + col] : 0.f;
    }
  };
  auto col_sum = [&]() {
    if (csum_on)
#pragma unroll
      for (int q = 0; q < 8; ++q) csum += va[q];
  };
  auto sstore = [&](int buf) {
    if (!stager) return;
    const int o = col * 4 + wg_slot(col, h);
    wg_bf16x8 p0, p1, p2;
    col_sum();
    wg_split(va, p0, p1, p2);
    L(buf, 0, 0)[o] = p0;
    L(buf, 0, 1)[o] = p1;
    L(buf, 0, 2)[o] = p2;
    wg_split(vx, p0, p1, p2);
    L(buf, 1, 0)[o] = p0;
    L(buf, 1, 1)[o] = p1;
    L(buf, 1, 2)[o] = p2;
  };
  const int g = lane >> 4, r16 = lane & 15;
  f32x4 acc[kSqW];
#pragma unroll
  for (int a = 0; a < kSqW; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  // stage(c): chunk c + 1 into the other buffer (its last readers, chunk c - 1's MFMAs, passed the
  // barrier), then chunk c + 2's loads; part 0 = the A item, 1 = the X item and the loads
  auto stage_part = [&](int c, int part_) {
    if (c + 1 >= nch) return;
    if constexpr ((DG & 2) != 0) return;
    if (!stager) return;
    const int buf = (c + 1) & 1, o = col * 4 + wg_slot(col, h);
    wg_bf16x8 p0, p1, p2;
    if (part_ == 0) col_sum();
    wg_split(part_ == 0 ? va : vx, p0, p1, p2);
    L(buf, part_, 0)[o] = p0;
    L(buf, part_, 1)[o] = p1;
    L(buf, part_, 2)[o] = p2;
    if (part_ == 1 && c + 2 < nch) gload(c + 2);
  };
  auto compute16 = [&](int c, auto typeb) {  // W16: the wave's tiles as described above (DG ignored)
    const int cur = c & 1;
    wg_bf16x8 fx[3], fa[3];
    auto mf = [&](f32x4& acc_) {
      f32x4 d = acc_;
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[2], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[1], d, 0, 0, 0);
      acc_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[0], d, 0, 0, 0);
    };
    if constexpr (!decltype(typeb)::value) {  // k tile wid, n tiles 0 .. 9
      const int cx = wid * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fx[pl] = L(cur, 1, pl)[cx * 4 + wg_slot(cx, g)];
#pragma unroll
      for (int a = 0; a < 10; ++a) {
        const int ca = a * 16 + r16;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fa[pl] = L(cur, 0, pl)[ca * 4 + wg_slot(ca, g)];
        mf(acc[a]);
      }
    } else {  // n tile wid - 3 (10 .. 12), k tiles 0 .. 12
      const int ca = (wid - 3) * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fa[pl] = L(cur, 0, pl)[ca * 4 + wg_slot(ca, g)];
#pragma unroll
      for (int a = 0; a < kSqW; ++a) {
        const int cx = a * 16 + r16;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fx[pl] = L(cur, 1, pl)[cx * 4 + wg_slot(cx, g)];
        mf(acc[a]);
      }
    }
  };
  auto compute = [&](int c) {
    const int cur = c & 1;
    wg_bf16x8 fx[3], fa[3];
    const int cx = wid * 16 + r16;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      if constexpr ((DG & 4) != 0)
        fx[pl] = __builtin_bit_cast(wg_bf16x8, f32x4{(float)(c + pl), 1.f, 2.f, 3.f});
      else
        fx[pl] = L(cur, 1, pl)[cx * 4 + wg_slot(cx, g)];
    }
#pragma unroll
    for (int a = 0; a < kSqW; ++a) {
      const int ca = a * 16 + r16;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        if constexpr ((DG & 4) != 0)
          fa[pl] = __builtin_bit_cast(wg_bf16x8, f32x4{(float)(a + pl), 1.f, (float)c, 3.f});
        else
          fa[pl] = L(cur, 0, pl)[ca * 4 + wg_slot(ca, g)];
      }
      if constexpr ((DG & 1) != 0) {
        acc[a] += __builtin_bit_cast(f32x4, fa[0]) + __builtin_bit_cast(f32x4, fx[1]);
        continue;
      }
      f32x4 d = acc[a];
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[2], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fx[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[1], d, 0, 0, 0);
      acc[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fx[0], d, 0, 0, 0);
    }
  };
  if (nch > 0) {
    gload(0);
    sstore(0);
  }
  if (nch > 1) gload(1);
  __syncthreads();
  if constexpr (W16) {
    // one loop per wave kind (wave-uniform), so each is register-allocated alone; both meet the same barriers
    if (wid < kSqW) {
      for (int c = 0; c < nch; ++c) {
        compute16(c, std::false_type());
        stage_part(c, 0);
        stage_part(c, 1);
        __syncthreads();
      }
    } else {
      for (int c = 0; c < nch; ++c) {
        compute16(c, std::true_type());
        stage_part(c, 0);
        stage_part(c, 1);
        __syncthreads();
      }
    }
  } else {
    for (int c = 0; c < nch; ++c) {
      compute(c);
      // (issuing this staging between the last MFMA tiles instead measured the same: DeepFM training
      // tower backward 0.2955 vs 0.2975 ms per layer)
      stage_part(c, 0);
      stage_part(c, 1);
      __syncthreads();
    }
  }
  float* out = part + (int64_t)slice * N * K;
  if (W16 && wid >= kSqW) {
    const int n1 = n0 + (wid - 3) * 16;
#pragma unroll
    for (int a = 0; a < kSqW; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n1 + 4 * g + r, k = k0 + a * 16 + r16;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[a][r];
      }
  } else {
    const int k = k0 + wid * 16 + r16;
#pragma unroll
    for (int a = 0; a < (W16 ? 10 : kSqW); ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + a * 16 + 4 * g + r;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[a][r];
      }
  }
  if (csum_on) {  // block-uniform; the LDS image is free after the loop's last barrier
    float* red = reinterpret_cast<float*>(wlds);
    if (stager) red[h * kSqT + col] = csum;
    __syncthreads();
    if (h == 0 && a_ok)
      cpart[(int64_t)slice * N + n0 + col] = ((red[col] + red[kSqT + col]) + red[2 * kSqT + col]) + red[3 * kSqT + col];
  }
}

// out[i] (=, or += when accum) sum_s part[s][i]: a block covers 64 outputs with 4 wave-groups, group
// q summing slices q, q + 4, ...; the 4 group sums are added in fixed order (deterministic).
// Blocks past ceil(n / 64) reduce a second array the same way (n2 outputs of part2 into out2, "=" only):
// the dW's fused bias partials ride its launch instead of a launch of their own.
__global__ __launch_bounds__(256) void slice_reduce_kernel(int S, int64_t n, const float* __restrict__ part,
                                                           float* __restrict__ out, int accum, int64_t n2 = 0,
                                                           const float* __restrict__ part2 = nullptr,
                                                           float* __restrict__ out2 = nullptr) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t nb1 = (n + 63) / 64;
  int64_t blk = blockIdx.x;
  if (blk >= nb1) {  // block-uniform
    blk -= nb1;
    n = n2;
    part = part2;
    out = out2;
    accum = 0;
  }
  const int64_t i = blk * 64 + c;
  float v = 0.f;
  if (i < n)
    for (int sl = q; sl < S; sl += 4) v += part[(int64_t)sl * n + i];
  red[q][c] = v;
  __syncthreads();
  if (q == 0 && i < n) {
    const float t = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    out[i] = accum ? out[i] + t : t;
  }
}

// slice_reduce_kernel on float4s (n, n2 multiples of 4, 16-B aligned arrays): a block covers 256 outputs; each
// output sums the same slices in the same order (bitwise the scalar kernel), with a quarter of the load
// instructions (DeepFM training's dW reductions read 41-64 MB each)
__global__ __launch_bounds__(256) void slice_reduce4_kernel(int S, int64_t n, const float* __restrict__ part,
                                                            float* __restrict__ out, int accum, int64_t n2,
                                                            const float* __restrict__ part2, float* __restrict__ out2) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ f4 red[4][64];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  int64_t n4 = n / 4;
  const int64_t nb1 = (n4 + 63) / 64;
  int64_t blk = blockIdx.x;
  if (blk >= nb1) {  // block-uniform
    blk -= nb1;
    n4 = n2 / 4;
    part = part2;
    out = out2;
    accum = 0;
  }
  const f4* p4 = reinterpret_cast<const f4*>(part);
  const int64_t i = blk * 64 + c;
  f4 v = f4{0.f, 0.f, 0.f, 0.f};
  if (i < n4)
    for (int sl = q; sl < S; sl += 4) v += p4[(int64_t)sl * n4 + i];
  red[q][c] = v;
  __syncthreads();
  if (q == 0 && i < n4) {
    const f4 t = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    f4* o4 = reinterpret_cast<f4*>(out) + i;
    *o4 = accum ? *o4 + t : t;
  }
}

// Column sums over row slices: part[slice][n] = sum_{r in slice} w[r] * M[r][n]  (w null: 1).
// Bias gradients (sum over the batch of dPre) and the output-weight gradients (h^T dz).  A block
// covers 64 columns x one slice with 4 wave-groups over interleaved rows (coalesced 256-B rows).
__global__ __launch_bounds__(256) void colsum_kernel(int rows, int N, const float* __restrict__ M, int ldm,
                                                     const float* __restrict__ w, int rows_per_slice,
                                                     float* __restrict__ part) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int r0 = blockIdx.y * rows_per_slice, r1 = min(rows, r0 + rows_per_slice);
  float acc = 0.f;
  if (n < N) {
#pragma unroll 8
    for (int r = r0 + q; r < r1; r += 4) acc += w ? w[r] * M[(int64_t)r * ldm + n] : M[(int64_t)r * ldm + n];
  }
  red[q][c] = acc;
  __syncthreads();
  if (q == 0 && n < N) part[(int64_t)blockIdx.y * N + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }

int ensure_part(TrainState& T, int64_t n) {
  if (n <= T.cap_part) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());
  tfree(T.part2);
  int st = talloc(&T.part2, (size_t)n);
  if (st) return st;
  T.cap_part = n;
  return RMX_OK;
}

// out (N x K row-major) (= or +=) A[rows][lda](N columns)^T . X[rows][ldx](K columns); zg (split GEMM
// only, wgrad_z_ok): X is the CIN outer product generated from x0 / up instead of read
bool wgrad_z_ok() { return f32_split_enabled() && tuning_get("wgrad_s3", 2) != 0; }

// bias (nullable): also bias[n] = sum_b A[b][n] when the kernel can fuse it (the 208 x 208 tile); *bias_done
// says whether it did (else the caller runs colsum)

// The 208 x 208 dW's slice count S (one block per CU): the multiple of 8 with the fewest rounds x chunks per
// block.  With smodel (knob "wgrad_smodel", default 1) the S partial planes the kernel writes and
// slice_reduce reads back are priced too (~8 B per output per slice at ~4 TB/s, against ~3.8 us per round of
// 32-row chunks): DeepFM training's layer-1 dW (624 x 400) took S = 128 (3 rounds x 16 chunks) and paid 33 us
// of slice reduction for it; without smodel rounds x chunks alone.  The two constants were measured on one
// MI355X and are fixed in the source, so S -- and with it the dW's fp32 summation order over the slices -- is
// a pure function of (rows, N, K, CU count): the same on every 256-CU MI355X, different on a part with
// another CU count (pinned for the bench shapes by tests/test_abi.py through
// rmx_debug_wgrad_slices).
int wgrad_sq_slices(int64_t rows, int N, int K, int tiles, int ncu, bool smodel) {
  ncu = std::max(ncu, 1);
  int S = 8;
  double best = -1.0;
  for (int s8 = 8; s8 <= 512; s8 += 8) {
    const int64_t chunks = round_up((rows + s8 - 1) / s8, kWgR) / kWgR;
    const int64_t rounds = ((int64_t)tiles * s8 + ncu - 1) / ncu;
    const double cost = smodel ? 3.8 * (double)(rounds * chunks) + (double)s8 * N * K * 8.0 / 4.0e6
                               : (double)(rounds * chunks);
    if (best < 0 || cost < best) {
      best = cost;
      S = s8;
    }
    if (chunks <= 1) break;
  }
  return S;
}

int wgrad(TrainState& T, hipStream_t s, int rows, int N, int K, const float* A, int lda, const float* X, int ldx,
          float* out, bool accum, const WgZ* zg = nullptr, float* bias = nullptr, bool* bias_done = nullptr) {
  if (bias_done) *bias_done = false;
  if (rows <= 0 || N <= 0 || K <= 0) return RMX_OK;
  // knob "wgrad_s3": 0 = the f32 MFMA kernel, 1 = split GEMM with 64 x 64 tiles, 2 = 128 x 128 tiles
  // default 2 since the single-buffered kernel (wgrad_sb): DeepFM training at B = 65,536 2.25 ->
  // 2.12 ms per step (on the double-buffered kernel the tower's dW, K <= 624, ran faster on 64 x 64)
  int var = f32_split_enabled() ? tuning_get("wgrad_s3", 2) : 0;
  // the generated CIN operand (N = H, K = F * Hp, rows = B * k) runs on the 128 x 128 tiles unless
  // "wgrad_gz" = 64: xDeepFM training at B = 4,096: CIN backward 14.88 -> 14.00 ms
  if (zg && var != 0) var = tuning_get("wgrad_gz", 128) == 64 ? 1 : 2;
  if (zg && !var) {
    set_error("wgrad: the generated CIN operand needs the split GEMM");
    return RMX_E_INVALID;
  }
  const WgZ z = zg ? *zg : WgZ{};
  // knob "wgrad_nk": the 208 x 128 tile in place of the 128 x 128 one -- 1 (default) for the CIN's
  // generated operand (xDeepFM training at B = 4,096: CIN backward 9.49 -> 8.73 ms), 2 for every dW
  // (the tower's 400 x 400 / 624 dW ran slower on it: DeepFM training 1.95 -> 2.19 ms), 0 off
  const int nkv = tuning_get("wgrad_nk", 1);
  const bool nk = var == 2 && (nkv == 2 || (nkv == 1 && zg));
  // knob "wgrad_sq": 1 (default) the 208 x 208 tile for a read (not generated) X, 0 off (DeepFM
  // training at B = 65,536: tower backward 0.346 / 0.346 / 0.445 -> 0.300 / 0.300 / 0.423 ms per layer,
  // 33.4 -> 35.4 M examples/s, profiles/r03/ab_wgrad_sq.txt)
  // (one block per CU: at small batches -- xDeepFM training, B = 4,096 -- the 128 x 128 tiles' two blocks
  // per CU win: tower layer-1 backward 0.083 vs 0.104 ms)
  // knob "wgrad_sq_gz": 1 the 208 x 208 tile also for the CIN's generated operand (else the 208 x 128 one)
  const bool sq_gz = zg && var == 2 && tuning_get("wgrad_sq_gz", 0) != 0 && rows >= 32768;
  const bool sq = sq_gz || (var == 2 && !zg && !nk && tuning_get("wgrad_sq", 1) != 0 && rows >= 32768);
  const int TT = var == 2 ? 128 : kWgT;
  const int tiles = sq ? ((N + kSqT - 1) / kSqT) * ((K + kSqT - 1) / kSqT)
                  : nk ?  ((N + kNkN - 1) / kNkN) * ((K + kNkK - 1) / kNkK)
                         : ((N + TT - 1) / TT) * ((K + TT - 1) / TT);
  // slices of ~1024 rows (one slice of both operands, (N + K) * 4 KiB, stays in an XCD's 4 MiB L2),
  // at least ~1024 blocks in flight, S a multiple of the 8 XCDs
  int S = std::max((rows + 1023) / 1024, std::min((1024 + tiles - 1) / tiles, std::max(1, rows / 64)));
  S = round_up(std::min(S, 512), 8);
  if (sq) {
    int ncu = 0, dev = 0;
    RMX_HIP(hipGetDevice(&dev));
    RMX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    S = wgrad_sq_slices(rows, N, K, tiles, ncu, tuning_get("wgrad_smodel", 1) != 0);
  }
  const int rps = round_up((rows + S - 1) / S, var ? kWgR : 16);
  const bool fuse_bias = sq && bias && tuning_get("wgrad_bias", 1) != 0;
  int st = ensure_part(T, (int64_t)S * N * K + (fuse_bias ? (int64_t)S * N : 0));
  if (st) return st;
  if (sq) {
    const size_t lds = sizeof(wg_bf16x8) * 2 * 2 * 3 * kSqT * 4;  // 156 KiB
    // (set at every launch, as launch_cfg does: a process may drive several devices)
    RMX_HIP(hipFuncSetAttribute(zg ? (const void*)wgrad_sq_kernel<true> : (const void*)wgrad_sq_kernel<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    float* cpart = fuse_bias ? T.part2 + (int64_t)S * N * K : nullptr;
#if RMX_WGRAD_SQ_DIAG
    const int dg = zg ? 0 : tuning_get("wgrad_diag", 0);  // timing probes (results wrong): DESIGN.md §10
#else
    const int dg = 0;
#endif
    // knob "wgrad_sq16": 16 waves balanced over the SIMDs (read operands only)
    const bool w16 = !zg && dg == 0 && tuning_get("wgrad_sq16", 1) != 0;
    if (w16) {
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_sq_kernel<false, 0, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL((wgrad_sq_kernel<false, 0, true>), dim3(tiles * S), dim3(kSq16Thr), lds, s, rows, N, K, A, lda,
                         X, ldx, rps, tiles, T.part2, cpart, z);
    } else if (zg)
      hipLaunchKernelGGL(wgrad_sq_kernel<true>, dim3(tiles * S), dim3(kSqThr), lds, s, rows, N, K, A, lda, X, ldx, rps,
                         tiles, T.part2, cpart, z);
#if RMX_WGRAD_SQ_DIAG
#define RMX_WG_DG(V)                                                                                              \
    else if (dg == V) {                                                                                           \
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_sq_kernel<false, V>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds));                                                                     \
      hipLaunchKernelGGL((wgrad_sq_kernel<false, V>), dim3(tiles * S), dim3(kSqThr), lds, s, rows, N, K, A, lda, X,   \
                         ldx, rps, tiles, T.part2, cpart, z);                                                     \
    }
    RMX_WG_DG(1) RMX_WG_DG(2) RMX_WG_DG(3) RMX_WG_DG(4) RMX_WG_DG(6)
#undef RMX_WG_DG
#endif
    else
      hipLaunchKernelGGL(wgrad_sq_kernel<false>, dim3(tiles * S), dim3(kSqThr), lds, s, rows, N, K, A, lda, X, ldx, rps,
                         tiles, T.part2, cpart, z);
    RMX_HIP(hipGetLastError());
    // the bias partials (fuse_bias) in the same launch: its blocks past the dW's
    const int64_t nb1 = ((int64_t)N * K + 63) / 64, nb2 = fuse_bias ? (N + 63) / 64 : 0;
    auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    const int64_t NK = (int64_t)N * K;
    if (NK % 4 == 0 && a16(T.part2) && a16(out) && (!fuse_bias || (N % 4 == 0 && a16(cpart) && a16(bias))) &&
        tuning_get("slice_reduce4", 1) != 0) {
      // (knob "slice_reduce4": the float4 form, default on)
      const int64_t b1 = (NK / 4 + 63) / 64, b2 = fuse_bias ? (N / 4 + 63) / 64 : 0;
      hipLaunchKernelGGL(slice_reduce4_kernel, dim3((unsigned)(b1 + b2)), dim3(256), 0, s, S, NK, T.part2, out,
                         accum ? 1 : 0, fuse_bias ? (int64_t)N : 0, cpart, bias);
    } else {
      hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)(nb1 + nb2)), dim3(256), 0, s, S, NK, T.part2, out,
                         accum ? 1 : 0, fuse_bias ? (int64_t)N : 0, cpart, bias);
    }
    RMX_HIP(hipGetLastError());
    if (fuse_bias) *bias_done = true;
    return RMX_OK;
  }
  // knob "wgrad_sb": 1 (default) the single-buffered kernel on the 128 x 128 tiles (two blocks per CU),
  // 2 also on the 64 x 64 tiles, 0 off
  if (nk) {
    const size_t lds = sizeof(wg_bf16x8) * 3 * (kNkN + kNkK) * 4;  // 63 KiB: two blocks per CU
    static bool attr = false;
    if (!attr) {
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_nk_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_nk_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
      attr = true;
    }
    if (zg)
      hipLaunchKernelGGL(wgrad_nk_kernel<true>, dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda, X, ldx, rps,
                         tiles, T.part2, z);
    else
      hipLaunchKernelGGL(wgrad_nk_kernel<false>, dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda, X, ldx, rps,
                         tiles, T.part2, z);
  } else if (var == 2 && tuning_get("wgrad_sb", 1) != 0) {
    const size_t lds = sizeof(wg_bf16x8) * 2 * 3 * 128 * 4;  // 48 KiB
    if (zg)
      hipLaunchKernelGGL((wgrad_s3_kernel<128, true, true>), dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda, X,
                         ldx, rps, tiles, T.part2, z);
    else
      hipLaunchKernelGGL((wgrad_s3_kernel<128, false, true>), dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda,
                         X, ldx, rps, tiles, T.part2, z);
  } else if (var == 2) {
    const size_t lds = sizeof(wg_bf16x8) * 2 * 2 * 3 * 128 * 4;
    static bool attr = false;
    if (!attr) {
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_s3_kernel<128, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      RMX_HIP(hipFuncSetAttribute((const void*)wgrad_s3_kernel<128, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr = true;
    }
    if (zg)
      hipLaunchKernelGGL((wgrad_s3_kernel<128, true>), dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda, X, ldx,
                         rps, tiles, T.part2, z);
    else
      hipLaunchKernelGGL((wgrad_s3_kernel<128, false>), dim3(tiles * S), dim3(512), lds, s, rows, N, K, A, lda, X,
                         ldx, rps, tiles, T.part2, z);
  } else if (var && tuning_get("wgrad_sb", 1) == 2) {  // 2: the 64 x 64 tiles single-buffered too
    const size_t lds = sizeof(wg_bf16x8) * 2 * 3 * 64 * 4;
    if (zg)
      hipLaunchKernelGGL((wgrad_s3_kernel<64, true, true>), dim3(tiles * S), dim3(256), lds, s, rows, N, K, A, lda, X,
                         ldx, rps, tiles, T.part2, z);
    else
      hipLaunchKernelGGL((wgrad_s3_kernel<64, false, true>), dim3(tiles * S), dim3(256), lds, s, rows, N, K, A, lda, X,
                         ldx, rps, tiles, T.part2, z);
  } else if (var) {
    const size_t lds = sizeof(wg_bf16x8) * 2 * 2 * 3 * 64 * 4;
    if (zg)
      hipLaunchKernelGGL((wgrad_s3_kernel<64, true>), dim3(tiles * S), dim3(256), lds, s, rows, N, K, A, lda, X, ldx,
                         rps, tiles, T.part2, z);
    else
      hipLaunchKernelGGL((wgrad_s3_kernel<64, false>), dim3(tiles * S), dim3(256), lds, s, rows, N, K, A, lda, X,
                         ldx, rps, tiles, T.part2, z);
  } else {
    hipLaunchKernelGGL(wgrad_kernel, dim3(tiles * S), dim3(256), 0, s, rows, N, K, A, lda, X, ldx, rps, tiles,
                       T.part2);
  }
  RMX_HIP(hipGetLastError());
  hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)(((int64_t)N * K + 63) / 64)), dim3(256), 0, s, S,
                     (int64_t)N * K, T.part2, out, accum ? 1 : 0);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// out[n] (= or +=) sum_r w[r] M[r][n]  (w null: plain column sums)
int colsum(TrainState& T, hipStream_t s, int rows, int N, const float* M, int ldm, const float* w, float* out,
           bool accum) {
  if (rows <= 0 || N <= 0) return RMX_OK;
  int S = std::max(1, std::min(128, rows / 512));
  const int rps = (rows + S - 1) / S;
  S = (rows + rps - 1) / rps;
  int st = ensure_part(T, (int64_t)S * N);
  if (st) return st;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64, S), dim3(256), 0, s, rows, N, M, ldm, w, rps, T.part2);
  RMX_HIP(hipGetLastError());
  hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, S, (int64_t)N, T.part2,
                     out, accum ? 1 : 0);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// output columns of a tower layer that belong to the layer (DCN fused extra columns excluded)
inline int eff_n(const DenseLayer& L) { return L.N1 >= 0 ? L.N1 : L.N; }

int ensure_train(rmx_model& m, int B) {
  if (!m.train) m.train = new TrainState();
  TrainState& T = *m.train;
  if (B <= T.B) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());
  tfree(T.x);
  for (auto& p : T.h) tfree(p);
  T.h.clear();
  for (size_t i = 1; i < T.hm.size(); ++i) tfree(T.hm[i]);  // (hm[0] is borrowed from fms, never owned)
  T.hm.clear();
  T.hm_ok.clear();
  tfree(T.g[0]);
  tfree(T.g[1]);
  tfree(T.fms);
  tfree(T.p);
  tfree(T.dz);
  tfree(T.ones);
  tfree(T.tmp);
  tfree(T.xcol);
  tfree(T.wc);
  tfree(T.coef);
  tfree(T.cst);
  tfree(T.gwc);
  for (auto& p : T.u) tfree(p);
  T.u.clear();
  tfree(T.x0);
  tfree(T.gx0);
  tfree(T.gu[0]);
  tfree(T.gu[1]);
  tfree(T.gpre);
  tfree(T.dzr);
  tfree(T.zb);
  tfree(T.onesR);
  tfree(T.part2);
  T.cap_part = 0;
  if (T.part) (void)hipFree(T.part);
  T.part = nullptr;
  int st;
  T.ldx = m.layers.empty() ? 0 : m.layers[0].Kpad;
  int maxld = std::max(T.ldx, 16);
  if (!m.layers.empty() && (st = talloc(&T.x, (size_t)B * T.ldx))) return st;
  for (auto& L : m.layers) {
    T.h.push_back(nullptr);
    if ((st = talloc(&T.h.back(), (size_t)B * L.Npad))) return st;
    T.hm.push_back(nullptr);
    T.hm_ok.push_back(0);
    // (layer 1's bits, from the training head, live in T.fms's second half)
    if (T.h.size() > 1 && L.N == 400 && L.Npad == 416 && (st = talloc(&T.hm.back(), (size_t)B * 16))) return st;
    maxld = std::max(maxld, L.Npad);
  }
  if (!m.layers.empty()) {
    if ((st = talloc(&T.g[0], (size_t)B * maxld))) return st;
    if ((st = talloc(&T.g[1], (size_t)B * maxld))) return st;
  }
  if ((st = talloc(&T.p, B)) || (st = talloc(&T.dz, B)) || (st = talloc(&T.ones, B))) return st;
  // [2][B][16]: the FM sums, then (training head, k_head_s3.hip XS) h1's ReLU mask bits
  if (m.type == RMX_MODEL_DEEPFM && m.k == 16 && (st = talloc(&T.fms, (size_t)B * 32))) return st;
  if ((st = talloc(&T.tmp, std::max(maxld, 2 * m.cross_depth + 1)))) return st;
  if (m.type == RMX_MODEL_XDEEPFM) {
    const int64_t R = (int64_t)B * m.k;
    int maxH = 16, maxFH = 16;
    for (auto& c : m.cin_layers) {
      maxH = std::max(maxH, c.Npad);
      maxFH = std::max(maxFH, std::max(m.F * c.Hp, c.NTpad));  // dz rows are NTpad wide (split GEMM)
    }
    for (auto& c : m.cin_layers) {
      T.u.push_back(nullptr);
      if ((st = talloc(&T.u.back(), (size_t)R * c.Npad))) return st;
    }
    const int64_t budget = 64ll << 20;  // floats of the Z chunk (256 MB)
    T.rc = (int)std::min<int64_t>(R, std::max<int64_t>(m.k, budget / maxFH / m.k * m.k));
    if ((st = talloc(&T.x0, (size_t)R * m.F)) || (st = talloc(&T.gx0, (size_t)R * m.F)) ||
        (st = talloc(&T.gu[0], (size_t)R * maxH)) || (st = talloc(&T.gu[1], (size_t)R * maxH)) ||
        (st = talloc(&T.gpre, (size_t)R * maxH)) || (st = talloc(&T.dzr, R)) ||
        (st = talloc(&T.zb, (size_t)T.rc * maxFH)) || (st = talloc(&T.onesR, R)))
      return st;
    hipLaunchKernelGGL(fill_kernel, dim3(nblk(R)), dim3(256), 0, m.ctx->stream, (int)R, 1.0f, T.onesR);
    RMX_HIP(hipGetLastError());
  }
  if (m.type == RMX_MODEL_DCN) {
    const int L = m.cross_depth, D = m.F * m.k;
    if ((st = talloc(&T.xcol, (size_t)B * (L + 1))) || (st = talloc(&T.wc, (size_t)(L + 1) * D)) ||
        (st = talloc(&T.coef, (size_t)B * (L + 1))) || (st = talloc(&T.cst, (size_t)B * (2 * L + 1))) ||
        (st = talloc(&T.gwc, (size_t)(L + 1) * D)))
      return st;
  }
  if (hipMalloc(&T.part, sizeof(double) * 2 * kMaxParts) != hipSuccess) {
    set_error("backward: out of device memory");
    return RMX_E_NOMEM;
  }
  hipLaunchKernelGGL(fill_kernel, dim3(nblk(B)), dim3(256), 0, m.ctx->stream, B, 1.0f, T.ones);
  RMX_HIP(hipGetLastError());
  T.B = B;
  return RMX_OK;
}

}  // namespace

void train_release(rmx_model& m) {
  if (!m.train) return;
  TrainState& T = *m.train;
  (void)hipDeviceSynchronize();
  tfree(T.x);
  for (auto& p : T.h) tfree(p);
  for (size_t i = 1; i < T.hm.size(); ++i) tfree(T.hm[i]);  // (hm[0] is borrowed from fms, never owned)
  tfree(T.g[0]);
  tfree(T.g[1]);
  tfree(T.fms);
  tfree(T.p);
  tfree(T.dz);
  tfree(T.ones);
  tfree(T.tmp);
  tfree(T.xcol);
  tfree(T.wc);
  tfree(T.coef);
  tfree(T.cst);
  tfree(T.gwc);
  for (auto& p : T.u) tfree(p);
  tfree(T.x0);
  tfree(T.gx0);
  tfree(T.gu[0]);
  tfree(T.gu[1]);
  tfree(T.gpre);
  tfree(T.dzr);
  tfree(T.zb);
  tfree(T.onesR);
  tfree(T.part2);
  if (T.part) (void)hipFree(T.part);
  delete m.train;
  m.train = nullptr;
}

int model_train(rmx_model& m, hipStream_t s, const FwdInputs& in, const TrainOutputs& o) {
  const int B = in.B;
  const int t = m.type;
  if (m.precision != kF32) {
    set_error("backward: fp32 models only (rmx_model_set_precision(RMX_DTYPE_F32))");
    return RMX_E_INVALID;
  }
  if (t == RMX_MODEL_DCN && m.cross_depth > kMaxFusedCross) {
    set_error("backward: DCN crossDepth must be <= " + std::to_string(kMaxFusedCross));
    return RMX_E_INVALID;
  }
  if ((in.ld > 0 && in.ld != m.k) || in.wld > 1) {
    set_error("backward: line-row (strided) tables are forward-only");
    return RMX_E_INVALID;
  }
  if (B <= 0) return RMX_OK;
  int st = model_ensure_ws(m, B);  // y12 (first order + FM) lives in the inference workspace
  if (st) return st;
  if ((st = ensure_train(m, B))) return st;
  if (m.timing) ++m.timed_calls;
  TrainState& T = *m.train;
  const int F = m.F, k = m.k, D = F * k, Lc = m.cross_depth;

  // ---- forward with stored activations ----
  bool head_fused = false;  // the head, the BCE and the output layer's backward ran as head_train_kernel
  if (t == RMX_MODEL_LR) {
    StageTimer tm(m, s, "first_order_sigmoid");
    if (in.y1) st = launch_sigmoid_out(s, B, in.y1, in.beta, T.p);
    else st = launch_encoder(s, 2, B, in.ids, nullptr, in.wtab, in.dtype, F, 0, nullptr, &in.beta, T.p);
    if (st) return st;
  } else {
    const float* pre = nullptr;
    // DeepFM, k = 16: the encoder kernel that reads the rows for the FM also stores them as the tower
    // input x (knob "train_fuse_x": 1 (default) DeepFM, 2 also the first-order-only models, 0 off). One
    // pass over the random rows instead of two: DeepFM training 36.5 -> 37.7 M examples/s (encoder 0.069 +
    // gather_x 0.099 -> 0.105 ms); the first-order kernel does not read the rows otherwise, and fused it
    // measured 0.039 vs 0.020 + 0.013 ms (xDeepFM, B = 4,096), so 2 is not the default
    const int fxk = tuning_get("train_fuse_x", 1);
    const bool fuse_x = k == 16 && T.ldx == D && fxk != 0 &&
                        (t == RMX_MODEL_DEEPFM ||
                         (fxk == 2 && !in.y1 && t != RMX_MODEL_PNN && t != RMX_MODEL_DNN));
    float* xo = fuse_x ? T.x : nullptr;
    // DeepFM at a batch that fills the GPU: encoder + layer 1 as the row-owner head storing x and the FM sums
    // too (k_head_s3.hip XS; knob "train_head_s3", default 1)
    const bool head_x = t == RMX_MODEL_DEEPFM && fuse_x && !in.y1 && in.ids && in.dtype == kF32 && T.fms &&
                        tuning_get("train_emb_fused", 1) != 0 && tuning_get("train_head_s3", 1) != 0 &&
                        m.layers.size() > 1 && tower_head_s3_usable(m.layers[0], B, F, k, true);
    for (auto& ok : T.hm_ok) ok = 0;
    if (head_x) {
      StageTimer tm(m, s, "head_x");
      T.fms_valid = true;
      if ((st = launch_tower_head_s3(s, m.layers[0], B, F, in.ids, (const float*)in.table, 0, (const float*)in.wtab, 0,
                                     T.h[0], m.layers[0].Npad, m.y12, 1, T.x, T.ldx, T.fms)))
        return st;
      T.hm[0] = T.fms + (int64_t)B * 16;  // (not owned: see ensure_train)
      T.hm_ok[0] = 1;
      pre = m.y12;
    } else if (t == RMX_MODEL_DEEPFM) {
      StageTimer tm(m, s, fuse_x ? "encoder_fm_x" : "encoder_fm");
      // the FM sums for the fused embedding gradient (knob "train_emb_fused", default on)
      T.fms_valid = T.fms && k == 16 && tuning_get("train_emb_fused", 1) != 0;
      if ((st = launch_encoder(s, in.y1 ? 3 : 1, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr,
                               nullptr, 0, 0, xo, T.fms_valid ? T.fms : nullptr)))
        return st;
      pre = m.y12;
    } else if (t != RMX_MODEL_DNN) {
      if (!in.y1) {
        StageTimer tm(m, s, fuse_x ? "first_order_x" : "first_order");
        if ((st = launch_encoder(s, 0, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr, nullptr, 0, 0,
                                 xo)))
          return st;
      }
      pre = m.y12;
    }
    if (t == RMX_MODEL_PNN) {
      StageTimer tm(m, s, "product");
      if ((st = launch_product(s, B, F, k, in.ids, in.table, in.dtype, m.pairs, F * (F - 1) / 2, T.x, kF32, T.ldx)))
        return st;
    } else if (!fuse_x) {
      StageTimer tm(m, s, "gather_x");
      if ((st = launch_gather_x(s, B, F, k, in.ids, in.table, in.dtype, T.x, kF32, T.ldx))) return st;
    }
    if (t == RMX_MODEL_XDEEPFM) {
      const float* uprev = nullptr;
      for (size_t l = 0; l < m.cin_layers.size(); ++l) {
        StageTimer tm(m, s, l == 0 ? "cin_layer1" : (l == 1 ? "cin_layer2" : "cin_layer3+"));
        // last = false: every layer's maps are stored (the backward needs them)
        if ((st = launch_cin_layer(s, m.cin_layers[l], l == 0, false, B, F, k, in.ids, (const float*)in.table, uprev,
                                   T.u[l], m.rowdot)))
          return st;
        uprev = T.u[l];
      }
    }
    const float* A = T.x;
    int lda = T.ldx;
    static const char* names[] = {"tower_layer1", "tower_layer2", "tower_layer3", "tower_layer4+"};
    for (size_t i = head_x ? 1 : 0; i < m.layers.size(); ++i) {
      const DenseLayer& L = m.layers[i];
      if (i == 1 && head_x) {
        A = T.h[0];
        lda = m.layers[0].Npad;
      }
      StageTimer tm(m, s, names[std::min<size_t>(i, 3)]);
      XColArgs xc{T.xcol, L.N1, Lc + 1};
      const bool fused = i == 0 && m.dcn_fused;
      if (i > 0 && layer_s3_usable(L, false, B, lda, L.Npad)) {
        // 400 x 400 hidden layers: the row-owner kernel (k_layer_s3.hip; knob "train_layer_s3")
        uint32_t* hmi = reinterpret_cast<uint32_t*>(T.hm[i]);
        if ((st = launch_layer_s3(s, L, false, B, A, lda, T.h[i], L.Npad, hmi, nullptr))) return st;
        T.hm_ok[i] = hmi ? 1 : 0;
      } else if ((st = launch_tower_layer(s, L, B, A, lda, nullptr, T.h[i], L.Npad, Epi::kReluStore, nullptr,
                                          fused ? &xc : nullptr))) {
        return st;
      }
      A = T.h[i];
      lda = L.Npad;
    }
    OutArgs oa{};
    if (t == RMX_MODEL_DCN) {
      StageTimer tm(m, s, "cross");
      // wc = [w_0 .. w_{L-1}; W_out[0:D]]; the unfused case gets u / v from one GEMM
      RMX_HIP(hipMemcpyAsync(T.wc, m.cross_w, sizeof(float) * Lc * D, hipMemcpyDeviceToDevice, s));
      RMX_HIP(hipMemcpyAsync(T.wc + (int64_t)Lc * D, m.wo_x, sizeof(float) * D, hipMemcpyDeviceToDevice, s));
      if (!m.dcn_fused && (st = launch_gemm_f32(s, true, false, B, Lc + 1, D, T.x, T.ldx, T.wc, D, T.xcol, Lc + 1)))
        return st;
      if ((st = launch_cross_finish(s, B, Lc, T.xcol, m.cross_scalars, m.pre2))) return st;
      oa.pre2 = m.pre2;
    }
    if (t == RMX_MODEL_XDEEPFM) {
      oa.rowsum = m.rowdot;
      oa.rowsum_k = k;
    }
    oa.wo = m.wo;
    oa.bo = m.bo;
    oa.has_bo = m.has_bo ? 1 : 0;
    oa.pre = pre;
    oa.beta = in.beta;
    oa.out = T.p;
    const int Nh = eff_n(m.layers.back());
    head_fused = tuning_get("train_head_fused", 1) != 0 && Nh <= kHeadCols * 64;
    if (head_fused) {
      // logit + p + BCE + the output layer's dPre / dW_out in one pass over h (head_train_kernel)
      StageTimer tm(m, s, "head_bce");
      const int nparts = std::min(kMaxParts, (B + 15) / 16);  // >= 16 rows per block; 64 at B = 65,536
      const int per = (B + nparts - 1) / nparts;
      const int np = (B + per - 1) / per;
      float* cp = nullptr;
      // dW_out partials: np slices reduced in two fixed-order passes when np is a multiple of 16 (np / 16
      // slices of 16 * Nh, then 16 slices of Nh): a single pass over 1,024 slices ran on 7 blocks
      const int G = (np % 16 == 0 && np >= 64) ? 16 : 1;
      if (o.g_mats) {
        if ((st = ensure_part(T, (int64_t)np * Nh + (int64_t)G * Nh))) return st;
        cp = T.part2;
      }
      hipLaunchKernelGGL(head_train_kernel, dim3(np), dim3(256), 0, s, B, Nh, A, lda, oa, o.targets, T.dz, T.g[0],
                         m.layers.back().Npad, per, T.part, cp);
      RMX_HIP(hipGetLastError());
      float* gbo = (m.has_bo && o.g_mats) ? o.g_mats + m.bo_off : nullptr;
      hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(256), 0, s, np, B, T.part, o.loss, o.g_bias, gbo);
      RMX_HIP(hipGetLastError());
      if (cp && G > 1) {
        float* cp2 = cp + (int64_t)np * Nh;
        // (the float4 form when the arrays allow it: the same sums in the same order)
        const bool v4 = Nh % 4 == 0 && ((uintptr_t)cp2 & 15) == 0 && ((uintptr_t)(o.g_mats + m.wo_off) & 15) == 0 &&
                        tuning_get("slice_reduce4", 1) != 0;
        if (v4)
          hipLaunchKernelGGL(slice_reduce4_kernel, dim3((unsigned)(((int64_t)G * Nh / 4 + 63) / 64)), dim3(256), 0, s,
                             np / G, (int64_t)G * Nh, cp, cp2, 0, (int64_t)0, nullptr, nullptr);
        else
          hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)(((int64_t)G * Nh + 63) / 64)), dim3(256), 0, s, np / G,
                             (int64_t)G * Nh, cp, cp2, 0);
        RMX_HIP(hipGetLastError());
        if (v4)
          hipLaunchKernelGGL(slice_reduce4_kernel, dim3((unsigned)((Nh / 4 + 63) / 64)), dim3(256), 0, s, G, (int64_t)Nh,
                             cp2, o.g_mats + m.wo_off, 0, (int64_t)0, nullptr, nullptr);
        else
          hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)((Nh + 63) / 64)), dim3(256), 0, s, G, (int64_t)Nh, cp2,
                             o.g_mats + m.wo_off, 0);
        RMX_HIP(hipGetLastError());
      } else if (cp) {
        hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)((Nh + 63) / 64)), dim3(256), 0, s, np, (int64_t)Nh, cp,
                           o.g_mats + m.wo_off, 0);
        RMX_HIP(hipGetLastError());
      }
    } else {
      StageTimer tm(m, s, "tower_head");
      if ((st = launch_tower_head(s, B, Nh, A, lda, oa))) return st;
    }
  }

  // ---- loss, dL/dz, bias gradient ----
  if (!head_fused) {
    StageTimer tm(m, s, "bce");
    const int nparts = std::min(kMaxParts, (B + kRedThreads - 1) / kRedThreads);
    const int per = (B + nparts - 1) / nparts;
    hipLaunchKernelGGL(bce_kernel, dim3(nparts), dim3(kRedThreads), 0, s, B, T.p, o.targets, T.dz, per, T.part);
    RMX_HIP(hipGetLastError());
    float* gbo = (m.has_bo && o.g_mats) ? o.g_mats + m.bo_off : nullptr;  // output Linear bias: same sum
    hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(256), 0, s, nparts, B, T.part, o.loss, o.g_bias, gbo);
    RMX_HIP(hipGetLastError());
  }
  if (o.g_w && t != RMX_MODEL_DNN && o.nnz > 0) {
    hipLaunchKernelGGL(w_grad_kernel, dim3(nblk(o.nnz)), dim3(256), 0, s, o.nnz, F, o.index, T.dz, o.g_w);
    RMX_HIP(hipGetLastError());
  }
  if (t == RMX_MODEL_LR) return RMX_OK;

  // ---- tower backward ----
  const int nl = (int)m.layers.size();
  if (!head_fused) {
    const DenseLayer& last = m.layers.back();
    const int N = eff_n(last);
    StageTimer tm(m, s, "head_back");
    if (o.g_mats && (st = colsum(T, s, B, N, T.h[nl - 1], last.Npad, T.dz, o.g_mats + m.wo_off, false))) return st;
    if (N % 4 == 0 && last.Npad % 4 == 0)
      hipLaunchKernelGGL(head_back4_kernel, dim3(nblk((int64_t)B * (N / 4))), dim3(256), 0, s, B, N / 4,
                         reinterpret_cast<const float4*>(T.h[nl - 1]), last.Npad / 4, T.dz,
                         reinterpret_cast<const float4*>(m.wo), reinterpret_cast<float4*>(T.g[0]), last.Npad / 4);
    else
      hipLaunchKernelGGL(head_back_kernel, dim3(nblk((int64_t)B * N)), dim3(256), 0, s, B, N, T.h[nl - 1], last.Npad,
                         T.dz, m.wo, T.g[0], last.Npad);
    RMX_HIP(hipGetLastError());
  }
  int cur = 0;
  bool emb_fused = false;  // layer 1's dX epilogue wrote the embedding gradient (DeepFM)
  static const char* bnames[] = {"tower_back1", "tower_back2", "tower_back3", "tower_back4+"};
  for (int l = nl - 1; l >= 0; --l) {
    const DenseLayer& L = m.layers[l];
    const int N = eff_n(L);
    StageTimer tm(m, s, bnames[std::min(l, 3)]);
    const float* xin = l == 0 ? T.x : T.h[l - 1];
    const int ldin = l == 0 ? T.ldx : m.layers[l - 1].Npad;
    const float* dpre = T.g[cur];
    float* dxin = T.g[cur ^ 1];
    const bool need_dx = l > 0 || o.g_emb || t == RMX_MODEL_DCN;
    // Linear blocks of this layer: (column range of x_in, W offset); PNN layer 1 = Linear(x) + Linear(ip)
    struct Blk { int c0, K; int64_t w; };
    Blk blks[2] = {{0, L.K, L.w_off}, {0, 0, -1}};
    int nb = 1;
    if (L.K1 >= 0) {
      blks[0] = {0, L.K1, L.w_off};
      blks[1] = {L.K1, L.K - L.K1, L.w_off2};
      nb = 2;
    }
    // dX on the split GEMM (W^T planes) when the layer has them, with the ReLU backward of the layer
    // below fused as a mask; otherwise gemm_f32_kernel + relu_back_kernel
    const float* mask = l > 0 ? T.h[l - 1] : nullptr;
    const int ldmask = l > 0 ? m.layers[l - 1].Npad : 0;
    bool masked = false, bias_done = false;
    for (int q = 0; q < nb; ++q) {
      const Blk& bk = blks[q];
      // (the bias gradient rides along with the first block's dW when the kernel fuses it)
      bool bd = false;
      if (o.g_mats && (st = wgrad(T, s, B, N, bk.K, dpre, L.Npad, xin + bk.c0, ldin, o.g_mats + bk.w, false, nullptr,
                                  (q == 0 && L.bias_mode == 1) ? o.g_mats + L.b_off : nullptr, &bd)))
        return st;
      bias_done = bias_done || bd;
      if (!need_dx) continue;
      if (nb == 1 && m.precision == kF32 && dx_s3_usable(L, ldin) && (!mask || L.NTpad <= ldmask)) {
        // DeepFM layer 1: dX + the FM term written straight as the embedding gradient (emb_grad_kernel's
        // arithmetic in the dX epilogue: dX is never stored and reread)
        emb_fused = l == 0 && t == RMX_MODEL_DEEPFM && T.fms_valid && o.g_emb && ldin == D && L.K == D;
        if (emb_fused) {
          const EmbGradArgs eg{T.x, T.fms, T.dz, T.ldx};
          if ((st = launch_dx_s3(s, L, B, dpre, L.Npad, o.g_emb, D, nullptr, 0, &eg))) return st;
        } else if (mask && T.hm_ok[l - 1] && bk.c0 == 0 && layer_s3_usable(L, true, B, L.Npad, ldin)) {
          // 400 x 400 layers whose lower layer left its mask bits: the row-owner kernel (k_layer_s3.hip)
          if ((st = launch_layer_s3(s, L, true, B, dpre, L.Npad, dxin, ldin, nullptr,
                                    reinterpret_cast<const uint32_t*>(T.hm[l - 1]))))
            return st;
        } else if ((st = launch_dx_s3(s, L, B, dpre, L.Npad, dxin + bk.c0, ldin, mask, ldmask))) {
          return st;
        }
        masked = mask != nullptr;
      } else {
        if ((st = launch_gemm_f32(s, false, false, B, bk.K, N, dpre, L.Npad, m.mats_dev + bk.w, bk.K, dxin + bk.c0,
                                  ldin)))
          return st;
      }
    }
    if (o.g_mats && L.bias_mode == 1 && !bias_done &&
        (st = colsum(T, s, B, N, dpre, L.Npad, nullptr, o.g_mats + L.b_off, false)))
      return st;
    if (o.g_mats && L.bias_mode == 2) {  // one CAdd(1) scalar over all outputs
      if ((st = colsum(T, s, B, N, dpre, L.Npad, nullptr, T.tmp, false))) return st;
      hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, s, N, T.tmp, o.g_mats + L.b_off);
      RMX_HIP(hipGetLastError());
    }
    if (l > 0 && !masked) {
      const DenseLayer& P = m.layers[l - 1];
      const int PN = eff_n(P);
      hipLaunchKernelGGL(relu_back_kernel, dim3(nblk((int64_t)B * PN)), dim3(256), 0, s, B, PN, T.h[l - 1], P.Npad,
                         dxin, P.Npad);
      RMX_HIP(hipGetLastError());
    }
    cur ^= 1;
  }
  float* dX = T.g[cur];  // dL/d(tower input) [B][ldx]

  // ---- DCN cross stack (closed form), adds into dX ----
  if (t == RMX_MODEL_DCN) {
    StageTimer tm(m, s, "cross_back");
    hipLaunchKernelGGL(cross_back_kernel, dim3(nblk(B)), dim3(256), 0, s, B, Lc, T.xcol, m.cross_scalars, T.dz,
                       T.coef, T.cst);
    RMX_HIP(hipGetLastError());
    // dX += coef [B][L+1] . wc [L+1][D]
    if ((st = launch_gemm_f32(s, false, true, B, D, Lc + 1, T.coef, Lc + 1, T.wc, D, dX, T.ldx))) return st;
    if (o.g_mats) {
      // gwc = coef^T x0 ; + the per-row constants summed over the batch ; beta_l sums
      if ((st = wgrad(T, s, B, Lc + 1, D, T.coef, Lc + 1, T.x, T.ldx, T.gwc, false))) return st;
      if ((st = colsum(T, s, B, 2 * Lc + 1, T.cst, 2 * Lc + 1, nullptr, T.tmp, false))) return st;
      hipLaunchKernelGGL(cross_wgrad_kernel, dim3(nblk((int64_t)(Lc + 1) * D)), dim3(256), 0, s, Lc, D, T.gwc, T.tmp,
                         o.g_mats + m.cross_w_off, o.g_mats + m.wo_x_off);
      RMX_HIP(hipGetLastError());
      hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, s, Lc, T.tmp + Lc + 1, o.g_mats + m.cross_b_off);
      RMX_HIP(hipGetLastError());
    }
  }

  // ---- xDeepFM CIN stack: gradients of C_l, c_l, W_out[pool slices] and dL/dx0 ----
  if (t == RMX_MODEL_XDEEPFM) {
    const int64_t R = (int64_t)B * k;
    StageTimer tm(m, s, "cin_back");
    hipLaunchKernelGGL(cin_x0_kernel, dim3(nblk(R * F)), dim3(256), 0, s, B, F, k, T.x, T.ldx, T.x0);
    RMX_HIP(hipGetLastError());
    hipLaunchKernelGGL(expand_dz_kernel, dim3(nblk(R)), dim3(256), 0, s, R, k, T.dz, T.dzr);
    RMX_HIP(hipGetLastError());
    RMX_HIP(hipMemsetAsync(T.gx0, 0, sizeof(float) * R * F, s));
    const int nc = (int)m.cin_layers.size();
    int gcur = 0;
    for (int l = nc - 1; l >= 0; --l) {
      const CinLayer& c = m.cin_layers[l];
      const int H = c.H, Hp = c.Hp, FH = F * Hp, ldu = c.Npad;
      const float* up = l == 0 ? T.x0 : T.u[l - 1];
      const int ldup = l == 0 ? F : m.cin_layers[l - 1].Npad;
      hipLaunchKernelGGL(cin_gpre_kernel, dim3(nblk(R * H)), dim3(256), 0, s, R, H, k, T.u[l], ldu,
                         l == nc - 1 ? nullptr : T.gu[gcur], T.dz, c.wo, T.gpre);
      RMX_HIP(hipGetLastError());
      if (o.g_mats) {
        // pooled slice of W_out: sum_r dz[b] u_l[r][h]; bias c_l: sum_r gpre[r][h]
        if ((st = colsum(T, s, (int)R, H, T.u[l], ldu, T.dzr, o.g_mats + c.wo_off, false))) return st;
        if ((st = colsum(T, s, (int)R, H, T.gpre, ldu, nullptr, o.g_mats + c.b_off, false))) return st;
      }
      // dC_l = gpre^T z over all rows, z = x0 (x) u_{l-1} generated inside the split wgrad (never stored)
      const bool genz = wgrad_z_ok();
      if (o.g_mats && genz) {
        WgZ zg;
        zg.x0 = T.x0;
        zg.up = up;
        zg.F = F;
        zg.Hp = Hp;
        zg.ldup = ldup;
        if ((st = wgrad(T, s, (int)R, H, FH, T.gpre, ldu, nullptr, 0, o.g_mats + c.w_off, false, &zg))) return st;
      }
      for (int64_t r0 = 0; r0 < R; r0 += T.rc) {
        const int rows = (int)std::min<int64_t>(T.rc, R - r0);
        const float* gp = T.gpre + r0 * ldu;
        if (o.g_mats && !genz) {  // f32 MFMA wgrad: z materialised per chunk
          hipLaunchKernelGGL(cin_z_kernel, dim3(nblk((int64_t)rows * FH)), dim3(256), 0, s, (int64_t)rows, F, Hp,
                             T.x0 + r0 * F, up + r0 * ldup, ldup, T.zb);
          RMX_HIP(hipGetLastError());
          if ((st = wgrad(T, s, rows, H, FH, gp, ldu, T.zb, FH, o.g_mats + c.w_off, r0 > 0))) return st;
        }
        // dL/dz for this chunk: gpre . C_l  [rows][F*Hp], on the split GEMM (C_l^T planes, row stride NTpad)
        if ((st = launch_cin_dz_s3(s, c, rows, gp, ldu, T.zb, c.NTpad))) return st;
        const int ldz = c.NTpad;
        // through u_{l-1} (layer 0: u_0 = x0, so into gx0 as well)
        float* gout = l == 0 ? T.gx0 + r0 * F : T.gu[gcur ^ 1] + r0 * m.cin_layers[l - 1].Npad;
        const int ldo = l == 0 ? F : m.cin_layers[l - 1].Npad;
        // knob "cin_back_fused" (default 1): both contractions in one pass over dL/dz
        const int vec = Hp % 4 == 0 ? 4 : 1;
        const size_t smem = sizeof(float) * ((size_t)F * (Hp / vec) + (size_t)(256 / std::max(1, Hp / vec)) * Hp);
        if (tuning_get("cin_back_fused", 1) && Hp / vec <= 256 && smem <= 64 * 1024) {
          if (vec == 4)
            hipLaunchKernelGGL(cin_back_fused_kernel<4>, dim3(rows), dim3(256), smem, s, (int64_t)rows, F, Hp, T.zb,
                               ldz, up + r0 * ldup, ldup, T.x0 + r0 * F, T.gx0 + r0 * F, gout, ldo, l == 0 ? 1 : 0);
          else
            hipLaunchKernelGGL(cin_back_fused_kernel<1>, dim3(rows), dim3(256), smem, s, (int64_t)rows, F, Hp, T.zb,
                               ldz, up + r0 * ldup, ldup, T.x0 + r0 * F, T.gx0 + r0 * F, gout, ldo, l == 0 ? 1 : 0);
          RMX_HIP(hipGetLastError());
        } else {
          hipLaunchKernelGGL(cin_back_x0_kernel, dim3(rows), dim3(256), 0, s, (int64_t)rows, F, Hp, T.zb, ldz,
                             up + r0 * ldup, ldup, T.gx0 + r0 * F);
          RMX_HIP(hipGetLastError());
          hipLaunchKernelGGL(cin_back_u_kernel, dim3(nblk((int64_t)rows * Hp)), dim3(256), 0, s, (int64_t)rows, F,
                             Hp, T.zb, ldz, T.x0 + r0 * F, gout, ldo, l == 0 ? 1 : 0);
          RMX_HIP(hipGetLastError());
        }
      }
      gcur ^= 1;
    }
  }

  // ---- embedding gradients ----
  if (o.g_emb && !emb_fused) {
    StageTimer tm(m, s, "emb_grad");
    if (t == RMX_MODEL_PNN)
      hipLaunchKernelGGL(pnn_emb_grad_kernel, dim3(nblk((int64_t)B * D)), dim3(256), 0, s, B, F, k, T.x, T.ldx, dX,
                         T.ldx, o.g_emb);
    else
      hipLaunchKernelGGL(emb_grad_kernel, dim3(nblk((int64_t)B * k)), dim3(256), 0, s, B, F, k, T.x, T.ldx, dX,
                         T.ldx, T.dz, t == RMX_MODEL_DEEPFM ? 1 : 0, t == RMX_MODEL_XDEEPFM ? T.gx0 : nullptr,
                       o.g_emb);
    RMX_HIP(hipGetLastError());
  }
  return RMX_OK;
}

}  // namespace rmx

extern "C" int rmx_debug_wgrad_slices(int64_t rows, int N, int K, int ncu) {
  if (rows <= 0 || N <= 0 || K <= 0 || ncu <= 0) {
    rmx::set_error("rmx_debug_wgrad_slices: rows, N, K and ncu must be positive");
    return RMX_E_INVALID;
  }
  const int tiles = ((N + rmx::kSqT - 1) / rmx::kSqT) * ((K + rmx::kSqT - 1) / rmx::kSqT);
  return rmx::wgrad_sq_slices(rows, N, K, tiles, ncu, rmx::tuning_get("wgrad_smodel", 1) != 0);
}
