// rmx_internal.hpp -- shared declarations of librmx (MI355X / gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rmx.h"

namespace rmx {

void set_error(const std::string& msg);
int tuning_get(const char* key, int def);  // rmx_set_tuning knobs (capi.hip)

#define RMX_HIP(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::rmx::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                       __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);     \
      return RMX_E_HIP;                                                            \
    }                                                                              \
  } while (0)

// ---------------------------------------------------------------- layers ----
// A BigDL Linear(in = K, out = N) packed for the fp32 MFMA GEMM:
//   W chunked as [Kpad/16][Npad][16] (each 16-wide K chunk of all N rows contiguous),
//   zero padded in K and N; bias [Npad] zero padded.
struct DenseLayer {
  int K = 0, N = 0, Kpad = 0, Npad = 0;
  int64_t w_off = -1;   // offset of W (out x in row-major) in mats
  int64_t b_off = -1;   // offset of bias in mats, -1 = none
  int K1 = -1;          // PNN: columns [0, K1) come from W at w_off (N x K1), [K1, K) from
  int64_t w_off2 = -1;  //      W2 at w_off2 (N x (K - K1)): Linear(x) + Linear(ip) as one GEMM
  int bias_mode = 1;    // 0 none, 1 per-output bias[N], 2 one scalar broadcast (CAdd(1))
  float* W = nullptr;   // device, packed
  float* b = nullptr;   // device [Npad]
};

constexpr int kChunk = 16;  // K chunk of the GEMM (= one field row at k = 16)

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------- kernels ---
// A operand producer for the first tower layer.
struct AGatherArgs {
  const int32_t* ids;  // [M][F] or nullptr (implicit id = m*F + f, the L-A path)
  const float* table;  // [rows][k]
  int F, k;
};

enum class Epi : int {
  kReluStore = 0,  // C = ReLU(acc + b), stored [M][ldc]
  kOutput = 1,     // logit = sum_n ReLU(acc + b)[n] * wo[n] (+ bo); combine + sigmoid
};

struct OutArgs {
  const float* wo;       // [Npad] output weights (zero padded), device
  float bo;              // output bias (0 when the output Linear has none)
  int has_bo;
  const float* pre;      // [M] term added before this one (y1+y2 for DeepFM, y1 ...), or null
  const float* pre2;     // [M] second additive term (DCN cross), or null
  const float* rowsum;   // [M*rowsum_k] per-row partials summed per sample (xDeepFM CIN), or null
  int rowsum_k;
  float beta;            // global bias
  float* out;            // [M] probabilities
};

int launch_tower_layer(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
                       const AGatherArgs* gather, float* C, int ldc, Epi epi, const OutArgs* oa);

int launch_encoder(hipStream_t s, int mode, int M, const int32_t* ids, const float* table,
                   const float* wtab, int F, int k, float* y, const float* beta, float* prob);
int launch_first_order_csr(hipStream_t s, int B, const int64_t* row_ptr, const float* w, float* y);
int launch_sigmoid_out(hipStream_t s, int B, const float* y, float beta, float* out);
int launch_gen_ids(hipStream_t s, uint64_t seed, int64_t row0, int B, int F, int64_t V, int32_t* ids);
int launch_fill_table(hipStream_t s, uint64_t seed, int64_t V, int k, float* w, float* emb);
int launch_gather(hipStream_t s, int64_t n, const int32_t* ids, const float* wtab,
                  const float* emb, int k, float* w_out, float* e_out);
int launch_pack_linear(hipStream_t s, const float* mats_dev, DenseLayer& L);
int launch_transpose_kmajor(hipStream_t s, const float* src_kv, int64_t V, int k, float* dst_vk);

}  // namespace rmx
