// rmx_models.hpp -- model / table / context objects behind the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

#include "rmx_internal.hpp"

struct rmx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
};

struct rmx_table {
  rmx_ctx* ctx = nullptr;
  int64_t V = 0;
  int k = 0;
  int dtype = 0;          // RMX_DTYPE_F32 / RMX_DTYPE_BF16 (elements of w and emb)
  void* w = nullptr;      // [V]     first-order weights (Angel "weights" row 0)
  void* emb = nullptr;    // [V][k]  embeddings, row-major (Angel "embedding" rows 0..k-1, transposed)
  // k = 16 tables with knob "table_lines" 1 (default 0): a [V][32] line copy (elements of dtype), row =
  // [emb 16 | w | pad 15] -- one 128-B memory line per id instead of a 64-B row line plus a separate weight
  // line (fp32), or one 64-B half line instead of a 32-B row line plus a weight line (bf16, round 5).
  // Rebuilt from emb / w by every upload / fill (rmx_table_refresh_lines after writes through
  // device_ptrs); read by the models whose every table access takes a row stride
  // (rmx::model_reads_lines).  Measured ~1 % SLOWER for DeepFM layer 1 at V = 1M (0.1851 vs 0.1829 ms,
  // two A/B pairs on one box): the weight lines it saves hit the Infinity Cache, so it is off.
  float* line = nullptr;   // (bf16 tables: bf16 elements)
};

namespace rmx {

struct TrainState;  // train.hip: backward workspace + rocBLAS handle

// One forward's inputs, already on the device.
struct FwdInputs {
  int B = 0;
  const int32_t* ids = nullptr;    // [B][F] or nullptr: implicit id = b*F + f (L-A path)
  const void* table = nullptr;     // [rows][k]  (elements of dtype)
  const void* wtab = nullptr;      // [rows]
  int dtype = 0;                   // kF32 / kBF16
  // row stride of `table` and stride of `wtab` in elements (0: k and 1).  ld = wld = 32 with
  // wtab = table + 16: [emb 16 | w | pad] line rows (a sharded partition read in place at one rank,
  // or a replicated table's line copy); only the models of rmx::model_reads_lines (model_forward checks)
  int ld = 0, wld = 0;
  const float* y1 = nullptr;       // precomputed first order (L-A irregular index) or nullptr
  float beta = 0.f;
  float* out = nullptr;            // [B]
};

// DCN cross stack scalars for the fused closed form (k_interact.hip cross_finish_kernel)
constexpr int kMaxFusedCross = 8;
struct CrossScalars {
  float wsum[kMaxFusedCross];  // sum_d w_l[d]
  float beta[kMaxFusedCross];  // beta_l
  float wo_sum;                // sum_d W_out[d], d < D
};

// CIN layer (xDeepFM): C_l (H x F*Hp) packed [Hp_pad/16][F][Npad][16], bias, output slice.
struct CinLayer {
  int Hp = 0, Hp_pad = 0, H = 0, Npad = 0;
  int64_t w_off = -1, b_off = -1, wo_off = -1;
  float* W = nullptr;
  float* b = nullptr;
  float* wo = nullptr;  // [Npad] slice of the output Linear for this layer's pooled maps
  bf16_t* W3 = nullptr;  // kPrecS3 planes of W (k_gemm_s3.hip), in the chunk-map K order when map_on
  // kPrecS3 K-chunk map (k_gemm.hpp cin_chunk): one entry f0 | hc << 16 | pair << 30 per 16-wide
  // chunk.  Layer 1 keeps only the h <= f half of its symmetric z = x0 (x) x0 (folded weights
  // C[f,h] + C[h,f]), and an h-chunk with <= 8 live maps carries two fields per chunk.
  int* cmap = nullptr;
  float* Wm = nullptr;  // fp32 [ncm][Npad][16] mapped weights (the split planes' source)
  int ncm = 0, tri = 0;
  int map_on = 0;       // W3 was packed in the mapped order (knob "cin_map" at set_mats)
  // backward dL/dz = gpre C_l on the split GEMM: C_l^T packed [KTpad/16][NTpad][16] (K = H, N = F Hp)
  float* WT = nullptr;
  bf16_t* WT3 = nullptr;
  int KTpad = 0, NTpad = 0;
};

}  // namespace rmx

struct rmx_model {
  rmx_ctx* ctx = nullptr;
  int type = 0;
  int64_t input_dim = 0;
  int F = 0, k = 0;
  std::vector<int> fc, cin;
  int cross_depth = 0;
  std::vector<int32_t> sizes;  // getMatsSize
  int64_t mats_len = 0;

  // ---- device parameters (packed from mats) ----
  float* mats_dev = nullptr;                // raw mats copy
  std::vector<rmx::DenseLayer> layers;      // tower; the last one runs the output head
  int64_t wo_off = -1, bo_off = -1;         // output Linear weights / bias in mats
  float* wo = nullptr;                      // device [Npad of last layer]
  float bo = 0.f;
  bool has_bo = false;
  std::vector<rmx::CinLayer> cin_layers;    // xDeepFM
  int64_t wo_cin_off = -1;                  // start of the pooled-CIN slice of W_out
  int64_t cross_w_off = -1, cross_b_off = -1, wo_x_off = -1;  // DCN
  float* cross_w = nullptr;                 // [L][D]
  float* cross_b = nullptr;                 // [L]
  float* wo_x = nullptr;                    // [D] slice of W_out for x_L
  bool dcn_fused = false;                   // cross dots fused into tower layer 1 (fcDims >= 2)
  rmx::CrossScalars cross_scalars{};
  float* xcol = nullptr;                    // [B][L + 1] raw fused cross dots
  int32_t* pairs = nullptr;                 // PNN (row, col) pairs [P][2]
  int precision = 0;                        // kF32 / kBF16 (rmx_model_set_precision)
  bool params_ready = false;
  float beta = 0.f;
  bool beta_set = false;

  // ---- workspace (grown on demand) ----
  int ws_B = 0;
  float* h[2] = {nullptr, nullptr};   // [B][Npad] tower activations
  float* y12 = nullptr;               // [B] first order (+ FM)
  float* pre2 = nullptr;              // [B] model-specific additive term (CIN / cross)
  float* xbuf = nullptr;              // [B][Kpad0] materialised A (PNN [x | ip], generic k)
  float* ubuf[2] = {nullptr, nullptr};  // [B*k][Npad] CIN maps
  float* rowdot = nullptr;            // [B*k] CIN per-row output partials
  float* opart = nullptr;             // [slices][B] partial logits of a column-sliced output layer
  // L-A staging
  int64_t la_nnz = 0;
  int la_B = 0;
  float* la_E = nullptr;
  float* la_w = nullptr;
  int64_t* la_rowptr = nullptr;
  float* la_out = nullptr;
  rmx::bf16_t* la_E16 = nullptr;                 // bf16 models: the rounded L-A arrays
  rmx::bf16_t* la_w16 = nullptr;
  int64_t la16_cap = 0;
  std::vector<int64_t> h_rowptr;
  std::vector<float> h_wperm;

  rmx::TrainState* train = nullptr;          // backward (train.hip), created on first use
  struct LaGrad {                            // L-A backward staging (rmx_backward), grown on demand
    int64_t nnz = 0, B = 0, ml = 0;
    float *gw = nullptr, *ge = nullptr, *gm = nullptr, *gb = nullptr, *tg = nullptr;
    int32_t* idx = nullptr;
  } la_grad;

  // ---- reentrancy (rmx.h "Threading"): one caller at a time; calls on different streams are
  //      ordered on the device by an event (rmx::ModelUse) ----
  std::mutex mu;
  hipStream_t ws_stream = nullptr;  // stream of the last call that used the workspace
  hipEvent_t ws_fence = nullptr;    // recorded on it at the end of that call (or, lazy, at the hand-over)
  bool ws_fence_lazy = false;       // the fence is not recorded yet: record it on ws_stream at the hand-over

  // ---- stage timing ----
  bool timing = false;
  int timed_calls = 0;
  std::vector<std::string> stage_names;
  std::vector<float> stage_ms;
  struct Pending { int stage; hipEvent_t a, b; };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> ev_pool;
};

namespace rmx {
int model_build(rmx_model& m);
void model_init_mats(const rmx_model& m, uint64_t seed, float* mats);
void model_release(rmx_model& m);
int model_load_mats(rmx_model& m, const float* host_mats, bool sync);
int model_set_precision(rmx_model& m, int dtype);
int model_forward(rmx_model& m, hipStream_t s, const FwdInputs& in);
// models whose every table read takes a row stride (DeepFM / DNN at k = 16, LR): they can read
// [emb | w | pad] line rows in place (FwdInputs::ld / wld)
bool model_reads_lines(const rmx_model& m);
// the forward's table operands: the line copy when the table has one and the model reads lines
void table_inputs(const rmx_table& t, const rmx_model& m, FwdInputs& in);
int table_refresh_lines(rmx_table& t);
int launch_pack_lines(hipStream_t s, int64_t V, const void* emb, const void* w, void* line, int dt);
int model_forward_host(rmx_model& m, int B, int64_t nnz, const int64_t* index, bool regular, bool sorted,
                       float bias, const float* weights, const float* embedding, const float* mats,
                       float* out);
int model_collect_timing(rmx_model& m);
int model_ensure_ws(rmx_model& m, int B);  // inference workspace (y12, h, ...) for batches <= B
int model_stage_host(rmx_model& m, int B, int64_t nnz, const int64_t* index, bool regular, bool sorted,
                     float bias, const float* weights, const float* embedding, const float* mats, FwdInputs* in);

// Backward (train.hip).  One training pass over a batch: forward with stored activations, BCE
// loss, and the gradients RecModel.backward writes back (all device pointers; g_w / g_emb may be
// null).  index: device int32 COO rows of the nnz weights (null: n / F).  loss: device [1].
struct TrainOutputs {
  const float* targets = nullptr;   // [B]
  const int32_t* index = nullptr;   // [nnz] or null
  int64_t nnz = 0;
  float* g_bias = nullptr;          // [1]
  float* g_w = nullptr;             // [nnz]
  float* g_emb = nullptr;           // [nnz * k]
  float* g_mats = nullptr;          // [mats_len]
  float* loss = nullptr;            // [1]
};
int model_train(rmx_model& m, hipStream_t s, const FwdInputs& in, const TrainOutputs& o);
void train_release(rmx_model& m);

// Serialises the callers of one model (its workspace, staging buffers and timing state are shared):
// the host lock is held for the whole call, and the call's last queued work is marked by an event;
// a call on another stream than the previous one first makes its stream wait for that event, so
// the previous call's kernels are done with the workspace before this call's run.  (The event is
// recorded at the end of every call, while the caller's stream is known to be alive.)
template <class T>
struct StreamUse {
  T& o;
  hipStream_t s;
  std::unique_lock<std::mutex> lk;
  int st = RMX_OK;
  // The fence is recorded lazily (round 6, knob "lazy_fence") for calls on the object's own context stream:
  // only when a later call arrives on another stream, on that context stream, under the lock -- it then
  // follows every operation the previous call enqueued there, which is all the hand-over needs.  Recorded
  // after every call, the marker sits between each pair of back-to-back launches.  A caller's own stream
  // keeps the eager record: it may be destroyed before the next call, the context's stream cannot be (the
  // object holds its context).
  bool lazy;
  StreamUse(T& oo, hipStream_t ss)
      : o(oo), s(ss), lk(oo.mu),
        lazy(oo.ctx && ss == oo.ctx->stream && tuning_get("lazy_fence", 0) != 0) {
    if (!o.ws_fence && hipEventCreateWithFlags(&o.ws_fence, hipEventDisableTiming) != hipSuccess) {
      o.ws_fence = nullptr;
      st = RMX_E_HIP;
    } else if (o.ws_stream && o.ws_stream != s) {
      if ((o.ws_fence_lazy && hipEventRecord(o.ws_fence, o.ws_stream) != hipSuccess) ||
          hipStreamWaitEvent(s, o.ws_fence, 0) != hipSuccess)
        st = RMX_E_HIP;
    }
    if (st) set_error("stream hand-over: HIP event create / wait failed");
  }
  ~StreamUse() {
    if (!o.ws_fence) return;
    if (lazy) {
      o.ws_stream = s;
      o.ws_fence_lazy = true;
    } else if (hipEventRecord(o.ws_fence, s) == hipSuccess) {
      o.ws_stream = s;
      o.ws_fence_lazy = false;
    }
  }
};
typedef StreamUse<rmx_model> ModelUse;

// Records HIP events around a stage on stream s when the model's timing is enabled.
struct StageTimer {
  rmx_model& m;
  hipStream_t s;
  int idx = -1;
  hipEvent_t a = nullptr;
  StageTimer(rmx_model& mm, hipStream_t ss, const char* name);
  ~StageTimer();
};
int shard_create(rmx_ctx* ctx, int64_t V, int k, int N, int rank, const void* unique_id, rmx_group* group,
                 rmx_shard** out);
int shard_destroy(rmx_shard* sh);

// kernels specific to the interaction encoders
int launch_pack_cin(hipStream_t s, const float* mats, int F, CinLayer& L);
std::vector<int> cin_chunk_map(int F, int Hp, bool tri);
int launch_pack_cin_map(hipStream_t s, const float* mats, int F, CinLayer& L);
int launch_pack_cin_t(hipStream_t s, const float* mats_dev, int F, CinLayer& c);
int launch_cin_dz_s3(hipStream_t s, const CinLayer& c, int rows, const float* gpre, int ldg, float* dz, int ldz);
int launch_cin_layer(hipStream_t s, const CinLayer& L, bool first, bool last, int B, int F, int k,
                     const int32_t* ids, const float* table, const float* u_prev, float* u_out,
                     float* rowdot, int ld = 0);
int launch_cross_finish(hipStream_t s, int B, int L, const float* xcol, const CrossScalars& cs, float* pre2);
int launch_cross(hipStream_t s, int B, int F, int k, int L, const int32_t* ids, const void* table, int dt,
                 const float* cross_w, const float* cross_b, const float* wo_x, float* pre2);
int launch_product(hipStream_t s, int B, int F, int k, const int32_t* ids, const void* table, int dt,
                   const int32_t* pairs, int P, void* xbuf, int xdt, int ldx);
int launch_gather_x(hipStream_t s, int B, int F, int k, const int32_t* ids, const void* table, int dt, void* xbuf,
                    int xdt, int ldx);
int tower_npad_for(int N);
// DeepFM's whole fp32 tower for small batches, one block per 16 samples (k_small_s3.hip)
bool tower_small_s3_usable(const rmx_model& m, int M, int F, int k, bool ids);
int launch_tower_small_s3(hipStream_t s, const rmx_model& m, int M, int F, const int32_t* ids, const float* table,
                          int ld, const float* wtab, int wld, const OutArgs& oa);
int cin_npad_for(int H);
}  // namespace rmx
