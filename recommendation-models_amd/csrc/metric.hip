// metric.hip -- device predict loop and AUC.
//
// predict: ParRecModel.predict* (yr/model/ParRecModel.scala:519-581) over a device-resident row
// set -- the forward of every batch, scores written in row order.
// AUC:     the metric the examples print every epoch (example/DeepFMLocalExample.scala:44-52,
// Angel's metric.AUC over (label, score) pairs; Angel is not in the reference tree, so the
// published definition is used: the Mann-Whitney statistic with tied scores counted 1/2).
//   1. sort (score, label) pairs by score (hipcub radix sort);
//   2. runs of equal scores (run-length encode) -> per-run sizes, positives per run (segmented sum);
//   3. AUC = sum_runs pos_g (neg_before_g + neg_g / 2) / (P N), in double, fixed reduction order.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rmx_models.hpp"

namespace rmx {
namespace {

__global__ void label_kernel(int64_t n, const float* __restrict__ labels, int* __restrict__ pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) pos[i] = labels[i] > 0.f ? 1 : 0;  // DeepFM.scala:106 (label > 0 -> positive)
}

__global__ void neg_kernel(int runs, const int* __restrict__ cnt, const int* __restrict__ pos,
                           int* __restrict__ neg) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < runs) neg[g] = cnt[g] - pos[g];
}

__global__ void widen_kernel(int n, const int* __restrict__ x, long long* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i];
}

// part[block] = sum over this block's runs of pos_g * (negbefore_g + 0.5 neg_g)  (doubles, tree)
__global__ __launch_bounds__(256) void auc_part_kernel(int runs, const int* __restrict__ pos,
                                                       const int* __restrict__ neg,
                                                       const long long* __restrict__ negbefore,
                                                       double* __restrict__ part) {
  __shared__ double sm[256];
  const int g = blockIdx.x * 256 + threadIdx.x;
  double v = 0.0;
  if (g < runs) v = (double)pos[g] * ((double)negbefore[g] + 0.5 * (double)neg[g]);
  sm[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sm[threadIdx.x] += sm[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sm[0];
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t n) {
    if (hipMalloc((void**)&p, sizeof(T) * (n ? n : 1)) != hipSuccess) {
      set_error("auc: out of device memory");
      return RMX_E_NOMEM;
    }
    return RMX_OK;
  }
};

int device_auc(hipStream_t s, int64_t n64, const float* labels, const float* scores, double* auc) {
  if (n64 > 2147483647ll) {
    set_error("rmx_auc: at most 2^31 - 1 pairs");
    return RMX_E_INVALID;
  }
  const int n = (int)n64;
  *auc = std::nan("");
  if (n == 0) return RMX_OK;
  DevBuf<int> lab, lab_s, cnt, posr, negr, nruns;
  DevBuf<float> key_s, uniq;
  DevBuf<int> off;
  DevBuf<long long> negb, negr64;
  DevBuf<double> part;
  int st;
  if ((st = lab.alloc(n)) || (st = lab_s.alloc(n)) || (st = key_s.alloc(n)) || (st = uniq.alloc(n)) ||
      (st = cnt.alloc(n + 1)) || (st = off.alloc(n + 1)) || (st = posr.alloc(n)) || (st = negr.alloc(n)) ||
      (st = negb.alloc(n)) || (st = negr64.alloc(n)) || (st = nruns.alloc(1)))
    return st;
  hipLaunchKernelGGL(label_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (int64_t)n, labels, lab.p);
  RMX_HIP(hipGetLastError());
  // temp storage: the largest requirement of the primitives below
  size_t tb = 0, t;
  RMX_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, t, scores, key_s.p, lab.p, lab_s.p, n, 0, 32, s));
  tb = std::max(tb, t);
  RMX_HIP(hipcub::DeviceRunLengthEncode::Encode(nullptr, t, key_s.p, uniq.p, cnt.p, nruns.p, n, s));
  tb = std::max(tb, t);
  RMX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t, cnt.p, off.p, n + 1, s));
  tb = std::max(tb, t);
  RMX_HIP(hipcub::DeviceSegmentedReduce::Sum(nullptr, t, lab_s.p, posr.p, n, off.p, off.p + 1, s));
  tb = std::max(tb, t);
  RMX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t, negr64.p, negb.p, n, s));
  tb = std::max(tb, t);
  DevBuf<unsigned char> tmp;
  if (hipMalloc(&tmp.p, tb ? tb : 1) != hipSuccess) {
    set_error("auc: out of device memory");
    return RMX_E_NOMEM;
  }
  t = tb;
  RMX_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, t, scores, key_s.p, lab.p, lab_s.p, n, 0, 32, s));
  t = tb;
  RMX_HIP(hipcub::DeviceRunLengthEncode::Encode(tmp.p, t, key_s.p, uniq.p, cnt.p, nruns.p, n, s));
  int runs = 0;
  RMX_HIP(hipMemcpyAsync(&runs, nruns.p, sizeof(int), hipMemcpyDeviceToHost, s));
  RMX_HIP(hipStreamSynchronize(s));
  // run offsets: exclusive scan of the run sizes with one trailing zero -> off[runs] = n
  RMX_HIP(hipMemsetAsync(cnt.p + runs, 0, sizeof(int), s));
  t = tb;
  RMX_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, t, cnt.p, off.p, runs + 1, s));
  t = tb;
  RMX_HIP(hipcub::DeviceSegmentedReduce::Sum(tmp.p, t, lab_s.p, posr.p, runs, off.p, off.p + 1, s));
  hipLaunchKernelGGL(neg_kernel, dim3((runs + 255) / 256), dim3(256), 0, s, runs, cnt.p, posr.p, negr.p);
  RMX_HIP(hipGetLastError());
  // negatives before each run (64-bit running count)
  hipLaunchKernelGGL(widen_kernel, dim3((runs + 255) / 256), dim3(256), 0, s, runs, negr.p, negr64.p);
  RMX_HIP(hipGetLastError());
  t = tb;
  RMX_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, t, negr64.p, negb.p, runs, s));
  const int nb = (runs + 255) / 256;
  if ((st = part.alloc(nb))) return st;
  hipLaunchKernelGGL(auc_part_kernel, dim3(nb), dim3(256), 0, s, runs, posr.p, negr.p, negb.p, part.p);
  RMX_HIP(hipGetLastError());
  std::vector<double> h(nb);
  RMX_HIP(hipMemcpyAsync(h.data(), part.p, sizeof(double) * nb, hipMemcpyDeviceToHost, s));
  RMX_HIP(hipStreamSynchronize(s));
  // P from the last exclusive-scan entry + last run, via one more small copy
  long long nb_last = 0;
  int neg_last = 0;
  RMX_HIP(hipMemcpyAsync(&nb_last, negb.p + (runs - 1), sizeof(long long), hipMemcpyDeviceToHost, s));
  RMX_HIP(hipMemcpyAsync(&neg_last, negr.p + (runs - 1), sizeof(int), hipMemcpyDeviceToHost, s));
  RMX_HIP(hipStreamSynchronize(s));
  const double N = (double)(nb_last + neg_last), P = (double)n - N;
  double sum = 0.0;
  for (double v : h) sum += v;  // fixed order
  if (P > 0 && N > 0) *auc = sum / (P * N);
  return RMX_OK;
}

}  // namespace
}  // namespace rmx

using namespace rmx;

extern "C" int rmx_predict_ids(rmx_model* m, const rmx_table* t, int64_t n_rows, const int32_t* d_ids, int32_t batch,
                               float* d_scores, void* stream) {
  if (!m || !t || !m->ctx || n_rows < 0 || batch <= 0 || (n_rows > 0 && (!d_ids || !d_scores))) {
    set_error("rmx_predict_ids: bad args");
    return RMX_E_INVALID;
  }
  if (!m->params_ready && m->mats_len > 0) {
    set_error("rmx_predict_ids: call rmx_model_set_mats first");
    return RMX_E_INVALID;
  }
  if (!m->beta_set) {
    set_error("rmx_predict_ids: call rmx_model_set_bias first");
    return RMX_E_INVALID;
  }
  if (m->type != RMX_MODEL_LR && (t->k != m->k || t->dtype != m->precision)) {
    set_error("rmx_predict_ids: table embedding_dim / dtype differ from the model");
    return RMX_E_SHAPE;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  ModelUse use(*m, s);
  if (use.st) return use.st;
  for (int64_t r0 = 0; r0 < n_rows; r0 += batch) {
    FwdInputs in;
    in.B = (int)std::min<int64_t>(batch, n_rows - r0);
    in.ids = d_ids + r0 * m->F;
    table_inputs(*t, *m, in);
    in.beta = m->beta;
    in.out = d_scores + r0;
    const int st = model_forward(*m, s, in);
    if (st) return st;
  }
  return RMX_OK;
}

extern "C" int rmx_auc(rmx_ctx* c, int64_t n, const float* d_labels, const float* d_scores, double* auc,
                       void* stream) {
  if (!c || !auc || n < 0 || (n > 0 && (!d_labels || !d_scores))) {
    set_error("rmx_auc: bad args");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(c->device));
  return device_auc(stream ? (hipStream_t)stream : c->stream, n, d_labels, d_scores, auc);
}
