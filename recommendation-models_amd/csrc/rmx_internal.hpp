// rmx_internal.hpp -- shared declarations of librmx (MI355X / gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rmx.h"

namespace rmx {

typedef __bf16 bf16_t;

// element types of tables / activations (include/rmx.h RMX_DTYPE_*)
constexpr int kF32 = 0, kBF16 = 1;

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
// four consecutive elements as fp32 (bf16 -> fp32 is exact)
__device__ __forceinline__ float4 load4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 load4(const bf16_t* p) {
  const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return (float)*p; }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = (bf16_t)v; }  // RNE (v_cvt_pk_bf16_f32)

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
  // DCN: extra output rows appended after the N1 layer rows, read raw (no bias / ReLU) by the
  // epilogue: rows [N1, N1 + nx) = the cross vectors w_l at w_off_x (nx x K), row N1 + nx = W_out[0:D]
  // at w_off_o.  N = N1 + nx + 1 then.  -1: none.
  int N1 = -1, nx = 0;
  int64_t w_off_x = -1, w_off_o = -1;
  float* W = nullptr;   // device, packed fp32 [Kpad/16][Npad][16]
  bf16_t* W16 = nullptr;  // device, packed bf16 [Kpad/32][Npad][32] (bf16 models; W unused then)
  bf16_t* W3 = nullptr;   // device, fp32 W split into 3 bf16 planes [ceil(Kpad/32)][3][Npad][32] (kPrecS3)
  // W^T for the backward's dX = dPre W on the split GEMM (fp32 single-block layers, train.hip):
  // a Linear(in = N, out = K) packed like W (fp32 [KTpad/16][NTpad][16]) and split into WT3
  int KTpad = 0, NTpad = 0;
  float* WT = nullptr;
  bf16_t* WT3 = nullptr;
  float* b = nullptr;   // device [Npad]
};

constexpr int kChunk = 16;  // K chunk of the GEMM (= one field row at k = 16)

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------- kernels ---
// A operand producer for the first tower layer.
struct AGatherArgs {
  const int32_t* ids;  // [M][F] or nullptr (implicit id = m*F + f, the L-A path)
  const float* table;  // [rows][ld] (bf16 elements for bf16 models: reinterpreted)
  int F, k;
  int ld;              // row stride in elements (0 = k); a power of two on k = 16 gathers (e.g. 32: the
                       // [emb 16 | w | pad] line rows of a sharded partition or a replicated line table)
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
  float* part;           // [Npad / BN][M] partial logits when the layer spans several column blocks
};

// Raw extra columns of a layer (DenseLayer::N1): written unrounded in fp32 to ptr[m * ld + (n - n_main)].
struct XColArgs {
  float* ptr;
  int n_main, ld;
};

// First order (+ DeepFM's FM) computed by tower layer 1 while its A rows stream through LDS
struct FmArgs {
  const void* w;   // first-order weights [V] (table element type)
  int w_bf16;      // 1: bf16 weights
  int sums;        // 1: y = y1 + y2 (DeepFM, split-GEMM layer 1); 0: y = y1
  int add;         // 1 (with sums): y already holds y1, y = y + y2
  float* y;        // [M]
  int wld;         // stride of the weights in elements (0 = 1; 32: the w slot of [emb | w | pad] line rows)
};

int launch_tower_layer(hipStream_t s, const DenseLayer& L, int M, const float* A, int lda,
                       const AGatherArgs* gather, float* C, int ldc, Epi epi, const OutArgs* oa,
                       const XColArgs* xc = nullptr, const FmArgs* fm = nullptr, bool cols32 = false);
// true when launch_tower_layer(L, M, gather, kReluStore) computes the FmArgs outputs (sums: + FM)
bool tower_fm_fusable(const DenseLayer& L, int M, const AGatherArgs* gather, bool sums);
// true when gathered layer 1 runs a 2-deep ring tile whose DMAs also carry the first-order weights
// (k_gemm.hpp kWRing): the first order is then summed from LDS at no cost
bool tower_wring(const DenseLayer& L, int M, const AGatherArgs* ga);

// bf16 tower tail (k_tail.hip): ReLU(H L2) -> ReLU(. L3) . wo -> head, one persistent launch, when
// both layers are bf16 with Npad = Kpad = 416; H [M][lda] bf16
bool tower_tail_usable(const DenseLayer& L2, const DenseLayer& L3, int M, int lda);
struct TailFirstOrder {  // the first order summed by the tail itself (bf16 weights)
  const int32_t* ids;    // [M][F]
  const bf16_t* w;       // weight of id at w[id * wld]
  int F, wld;
};
int launch_tower_tail_bf16(hipStream_t s, const DenseLayer& L2, const DenseLayer& L3, int M, const bf16_t* H, int lda,
                           const OutArgs& oa, const TailFirstOrder* fo = nullptr);
// fp32 tower layer 1 of DeepFM as a row-owner kernel (k_head_s3.hip): gather (k = 16, ids [M][F], table row
// of id at table + id * ld) + ReLU(x W1^T + b1) -> H [M][416] + first order (+ FM: fm_sums) -> fm_y [M]
bool tower_head_s3_usable(const DenseLayer& L1, int M, int F, int k, bool ids);
// one 400 x 400 fp32 layer as a row-owner kernel (k_layer_s3.hip), for the training step: forward
// (dx = false: C = ReLU(A W^T + b), and its ReLU mask bits hm_out [M][16]) or dX (dx = true: C = (A W) masked
// by the bits hm_in of the layer below, W^T's planes); A [M][lda], C [M][ldc]
bool layer_s3_usable(const DenseLayer& L, bool dx, int M, int lda, int ldc);
int launch_layer_s3(hipStream_t s, const DenseLayer& L, bool dx, int M, const float* A, int lda, float* C, int ldc,
                    uint32_t* hm_out, const uint32_t* hm_in);
// X / S (nullable; X non-null selects the training variant): also x [M][ldx], and into S [2][M][16] the FM
// sums, then h1's ReLU mask bits (k_rowown.hpp bits_set)
int launch_tower_head_s3(hipStream_t s, const DenseLayer& L1, int M, int F, const int32_t* ids, const float* table,
                         int ld, const float* wtab, int wld, float* H, int ldc, float* fm_y, int fm_sums,
                         float* X = nullptr, int ldx = 0, float* S = nullptr);
// DeepFM's whole fp32 tower in one persistent row-owner kernel (k_fused_s3.hip): gather (k = 16, ids [M][F])
// + first order + FM + three 400-wide split-GEMM layers + the head, h1 and h2 in registers -> oa.out [M]
bool tower_fused_s3_usable(const DenseLayer& L1, const DenseLayer& L2, const DenseLayer& L3, int M, int F, int k,
                           bool ids);
int launch_tower_fused_s3(hipStream_t s, const DenseLayer& L1, const DenseLayer& L2, const DenseLayer& L3, int M, int F,
                          const int32_t* ids, const float* table, int ld, const float* wtab, int wld,
                          const OutArgs& oa);
// fp32 tower tail (k_tail_s3.hip): ReLU(H L2) -> ReLU(. L3) . wo -> head on the split GEMM, one persistent
// launch, h2 in registers; both layers 400 x 400 with split planes; H [M][lda] fp32
bool tower_tail_s3_usable(const DenseLayer& L2, const DenseLayer& L3, int M, int lda);
int launch_tower_tail_s3(hipStream_t s, const DenseLayer& L2, const DenseLayer& L3, int M, const float* H, int lda,
                         const OutArgs& oa);
// logit / sigmoid head over stored last-hidden activations h[M][ldh] (one wave per row)
int launch_tower_head(hipStream_t s, int M, int N, const float* h, int ldh, const OutArgs& oa);
// ld: row stride of the table in elements (0 = k); wld: stride of the weights (0 = 1); xo (k = 16,
// modes 0 / 1 / 3): also write the gathered rows as fp32 x [M][F * 16] (the training forward's tower input);
// so (k = 16, modes 1 / 3): also write the FM sums s_j = sum_f e_fj as [M][16]
int launch_encoder(hipStream_t s, int mode, int M, const int32_t* ids, const void* table,
                   const void* wtab, int dt, int F, int k, float* y, const float* beta, float* prob, int ld = 0,
                   int wld = 0, float* xo = nullptr, float* so = nullptr);
int launch_first_order_csr(hipStream_t s, int B, const int64_t* row_ptr, const float* w, float* y);
int launch_sigmoid_out(hipStream_t s, int B, const float* y, float beta, float* out);
int launch_gen_ids(hipStream_t s, uint64_t seed, int64_t row0, int B, int F, int64_t V, int32_t* ids);
int launch_gen_ids_zipf(hipStream_t s, uint64_t seed, int64_t row0, int B, int F, int64_t V, double zs,
                        int32_t* ids);
int launch_fill_table(hipStream_t s, uint64_t seed, int64_t V, int k, void* w, void* emb, int dt);
int launch_gather(hipStream_t s, int64_t n, const int32_t* ids, const void* wtab,
                  const void* emb, int dt, int k, float* w_out, float* e_out);
int launch_convert_bf16(hipStream_t s, const float* src, int64_t n, bf16_t* dst);
int launch_widen_bf16(hipStream_t s, const bf16_t* src, int64_t n, float* dst);
int launch_pack_linear(hipStream_t s, const float* mats_dev, DenseLayer& L);
// W^T of a single-block layer into L.WT / L.WT3 (k_gemm_s3.hip)
int launch_pack_linear_t(hipStream_t s, const float* mats_dev, DenseLayer& L);
// dX[B][ldx] = dPre[B][lda] W (+ mask: dX *= (mask > 0)), on the split GEMM; RMX_E_INVALID when the
// layer has no W^T planes (the caller then uses its library GEMM)
// DeepFM: write dX of tower layer 1 as the embedding gradient (GemmArgs::eg_*)
struct EmbGradArgs {
  const float* x;   // [B][ldx] gathered rows
  const float* s;   // [B][16] FM sums
  const float* dz;  // [B] dL/dlogit
  int ldx;
};
int launch_dx_s3(hipStream_t s, const DenseLayer& L, int B, const float* dpre, int lda, float* dx, int ldx,
                 const float* mask, int ldmask, const EmbGradArgs* eg = nullptr);
bool dx_s3_usable(const DenseLayer& L, int ldx);
// fp32 packed [n16][Npad][16] -> the three bf16 planes of the split GEMM (k_gemm_s3.hip)
int launch_pack_split3(hipStream_t s, const float* Wp, int n16, int Npad, bf16_t* W3);
int64_t split3_elems(int n16, int Npad);  // bf16 elements of W3
// DeepFM's column-split small-batch path (models.hip, k_gemm_s3.hip p.cols32) up to this batch (knob "s3_cols"):
// B = 1,024 17.8 -> 19.2 M examples/s, but slower than the whole-tower kernel from B = 4,096 on
// (profiles/r06/ab_cols32.txt)
constexpr int kS3ColsMaxB = 2048;
bool f32_split_enabled();                 // rmx_set_tuning("f32_split") (default on)
// partial logits [ny][M] -> head combination + sigmoid
int launch_out_finish(hipStream_t s, int M, int ny, const OutArgs& oa);
int launch_transpose_kmajor(hipStream_t s, const float* src_kv, int64_t V, int k, void* dst_vk, int dt);

}  // namespace rmx
