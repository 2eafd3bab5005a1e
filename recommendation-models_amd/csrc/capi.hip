// capi.hip -- extern "C" entry points of librmx.so (see include/rmx.h).
//
// Host-side orchestration of the CTR forward: argument validation with the reference's
// failure modes, device parameter packing (mats -> MFMA-ready layers, once), workspace
// management, and the per-model kernel sequence.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rmx_internal.hpp"
#include "rmx_models.hpp"

namespace rmx {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

static std::mutex g_tune_mu;
static std::vector<std::pair<std::string, int>> g_tune;

int tuning_get(const char* key, int def) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  for (auto& kv : g_tune)
    if (kv.first == key) return kv.second;
  return def;
}

}  // namespace rmx

using namespace rmx;

// --------------------------------------------------------------------- misc --
extern "C" const char* rmx_last_error(void) { return g_err.c_str(); }
extern "C" int rmx_abi_version(void) { return RMX_ABI_VERSION; }

extern "C" int rmx_set_tuning(const char* key, int value) {
  if (!key) {
    set_error("rmx_set_tuning: key is NULL");
    return RMX_E_INVALID;
  }
  std::lock_guard<std::mutex> lk(g_tune_mu);
  for (size_t i = 0; i < g_tune.size(); ++i)
    if (g_tune[i].first == key) {
      if (value == RMX_TUNING_DEFAULT)
        g_tune.erase(g_tune.begin() + i);
      else
        g_tune[i].second = value;
      return RMX_OK;
    }
  if (value != RMX_TUNING_DEFAULT) g_tune.emplace_back(key, value);
  return RMX_OK;
}

extern "C" int rmx_get_tuning(const char* key, int def) { return key ? tuning_get(key, def) : def; }

#define CHECK_ARG(cond, msg)            \
  do {                                  \
    if (!(cond)) {                      \
      set_error(msg);                   \
      return RMX_E_INVALID;             \
    }                                   \
  } while (0)

// ------------------------------------------------------------------ context --
extern "C" int rmx_ctx_create(int device, rmx_ctx** out) {
  CHECK_ARG(out, "rmx_ctx_create: out is NULL");
  int n = 0;
  RMX_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) {
    set_error("rmx_ctx_create: no such device " + std::to_string(device));
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(device));
  auto* c = new rmx_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("rmx_ctx_create: hipStreamCreate failed");
    return RMX_E_HIP;
  }
  *out = c;
  return RMX_OK;
}

extern "C" int rmx_ctx_destroy(rmx_ctx* c) {
  if (!c) return RMX_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return RMX_OK;
}

extern "C" void* rmx_ctx_stream(rmx_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int rmx_stream_sync(void* s) {
  RMX_HIP(hipStreamSynchronize((hipStream_t)s));
  return RMX_OK;
}

extern "C" int rmx_malloc(rmx_ctx* c, size_t bytes, void** p) {
  CHECK_ARG(c && p, "rmx_malloc: bad args");
  RMX_HIP(hipSetDevice(c->device));
  if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) {
    set_error("rmx_malloc: out of device memory (" + std::to_string(bytes) + " bytes)");
    return RMX_E_NOMEM;
  }
  return RMX_OK;
}

extern "C" int rmx_free(rmx_ctx* c, void* p) {
  if (!p) return RMX_OK;
  if (c) RMX_HIP(hipSetDevice(c->device));
  RMX_HIP(hipFree(p));
  return RMX_OK;
}

extern "C" int rmx_memcpy_htod(rmx_ctx* c, void* dst, const void* src, size_t bytes) {
  CHECK_ARG(c, "rmx_memcpy_htod: ctx is NULL");
  RMX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  RMX_HIP(hipStreamSynchronize(c->stream));
  return RMX_OK;
}

extern "C" int rmx_memcpy_dtoh(rmx_ctx* c, void* dst, const void* src, size_t bytes) {
  CHECK_ARG(c, "rmx_memcpy_dtoh: ctx is NULL");
  RMX_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  RMX_HIP(hipStreamSynchronize(c->stream));
  return RMX_OK;
}

extern "C" int rmx_event_create(void** ev) {
  CHECK_ARG(ev, "rmx_event_create: NULL");
  hipEvent_t e;
  RMX_HIP(hipEventCreate(&e));
  *ev = (void*)e;
  return RMX_OK;
}
extern "C" int rmx_event_destroy(void* ev) {
  if (ev) RMX_HIP(hipEventDestroy((hipEvent_t)ev));
  return RMX_OK;
}
extern "C" int rmx_event_record(void* ev, void* s) {
  RMX_HIP(hipEventRecord((hipEvent_t)ev, (hipStream_t)s));
  return RMX_OK;
}
extern "C" int rmx_event_elapsed_ms(void* a, void* b, float* ms) {
  RMX_HIP(hipEventSynchronize((hipEvent_t)b));
  RMX_HIP(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return RMX_OK;
}

// -------------------------------------------------------------------- model --
extern "C" int rmx_model_create(rmx_ctx* c, int type, int64_t input_dim, int n_fields, int embedding_dim,
                                const int32_t* fc_dims, int n_fc, const int32_t* cin_dims, int n_cin,
                                int cross_depth, rmx_model** out) {
  CHECK_ARG(out, "rmx_model_create: bad args");  // ctx may be NULL: host-only model (metadata)
  if (type < RMX_MODEL_LR || type > RMX_MODEL_DNN) {
    set_error("rmx_model_create: unknown model type " + std::to_string(type));
    return RMX_E_TYPE;
  }
  std::unique_ptr<rmx_model> m(new rmx_model());
  m->ctx = c;
  m->type = type;
  m->input_dim = input_dim;
  m->F = n_fields;
  m->k = embedding_dim;
  if (fc_dims) m->fc.assign(fc_dims, fc_dims + std::max(n_fc, 0));
  if (cin_dims) m->cin.assign(cin_dims, cin_dims + std::max(n_cin, 0));
  m->cross_depth = cross_depth;
  const int st = model_build(*m);
  if (st != RMX_OK) return st;
  *out = m.release();
  return RMX_OK;
}

extern "C" int rmx_model_destroy(rmx_model* m) {
  if (!m) return RMX_OK;
  model_release(*m);
  delete m;
  return RMX_OK;
}

extern "C" int rmx_model_get_type(const rmx_model* m) { return m ? m->type : -1; }
extern "C" int64_t rmx_model_mats_len(const rmx_model* m) { return m ? m->mats_len : -1; }
extern "C" int64_t rmx_model_get_input_dim(const rmx_model* m) { return m ? m->input_dim : -1; }
extern "C" int rmx_model_get_embedding_dim(const rmx_model* m) {
  if (!m) return -1;
  return m->type == RMX_MODEL_LR ? -1 : m->k;  // LR.getEmbeddingDim = -1 (LR.scala:19)
}
extern "C" int rmx_model_get_mats_size(const rmx_model* m, int32_t* sizes, int cap, int* n) {
  CHECK_ARG(m && n, "rmx_model_get_mats_size: bad args");
  *n = (int)m->sizes.size();
  if (sizes)
    for (int i = 0; i < std::min(cap, *n); ++i) sizes[i] = m->sizes[i];
  return RMX_OK;
}

extern "C" int rmx_model_init_mats(const rmx_model* m, uint64_t seed, float* mats) {
  CHECK_ARG(m && (mats || m->mats_len == 0), "rmx_model_init_mats: bad args");
  model_init_mats(*m, seed, mats);
  return RMX_OK;
}

extern "C" int rmx_model_set_mats(rmx_model* m, const float* mats, int64_t n) {
  CHECK_ARG(m, "rmx_model_set_mats: model is NULL");
  CHECK_ARG(m->ctx, "rmx_model_set_mats: host-only model (created without a context)");
  if (m->mats_len > 0) CHECK_ARG(mats, "rmx_model_set_mats: mats is NULL");
  if (n != m->mats_len) {
    set_error("rmx_model_set_mats: mats has " + std::to_string(n) + " floats, getMatsSize needs " +
              std::to_string(m->mats_len));
    return RMX_E_MATS;
  }
  ModelUse use(*m, m->ctx->stream);  // in-flight calls on other streams still read the old weights
  if (use.st) return use.st;
  return model_load_mats(*m, mats, /*sync=*/true);
}

extern "C" int rmx_model_set_precision(rmx_model* m, int dtype) {
  CHECK_ARG(m, "rmx_model_set_precision: model is NULL");
  CHECK_ARG(m->ctx, "rmx_model_set_precision: host-only model (created without a context)");
  CHECK_ARG(dtype == RMX_DTYPE_F32 || dtype == RMX_DTYPE_BF16, "rmx_model_set_precision: dtype must be F32 or BF16");
  ModelUse use(*m, m->ctx->stream);
  if (use.st) return use.st;
  if (dtype == m->precision) return RMX_OK;
  if (dtype == RMX_DTYPE_BF16 && m->type == RMX_MODEL_XDEEPFM) {
    set_error("rmx_model_set_precision: the xDeepFM CIN runs in fp32 only");
    return RMX_E_INVALID;
  }
  return model_set_precision(*m, dtype);
}

extern "C" int rmx_model_set_bias(rmx_model* m, float bias) {
  CHECK_ARG(m, "rmx_model_set_bias: model is NULL");
  std::lock_guard<std::mutex> lk(m->mu);
  m->beta = bias;
  m->beta_set = true;
  return RMX_OK;
}

extern "C" int rmx_model_set_timing(rmx_model* m, int enable) {
  CHECK_ARG(m, "rmx_model_set_timing: model is NULL");
  std::lock_guard<std::mutex> lk(m->mu);
  m->timing = enable != 0;
  m->stage_names.clear();
  m->stage_ms.clear();
  m->timed_calls = 0;
  return RMX_OK;
}

extern "C" int rmx_model_get_timing(rmx_model* m, char* names, int name_stride, float* ms, int cap, int* n,
                                    int* calls) {
  CHECK_ARG(m && n, "rmx_model_get_timing: bad args");
  std::lock_guard<std::mutex> lk(m->mu);
  const int st = model_collect_timing(*m);
  if (st != RMX_OK) return st;
  *n = (int)m->stage_names.size();
  if (calls) *calls = m->timed_calls;
  for (int i = 0; i < std::min(cap, *n); ++i) {
    if (ms) ms[i] = m->stage_ms[i];
    if (names && name_stride > 0) {
      std::strncpy(names + (size_t)i * name_stride, m->stage_names[i].c_str(), name_stride - 1);
      names[(size_t)i * name_stride + name_stride - 1] = 0;
    }
  }
  return RMX_OK;
}

// -------------------------------------------------------------------- table --
static size_t dtype_size(int dt) { return dt == RMX_DTYPE_BF16 ? 2 : 4; }

extern "C" int rmx_table_create_ex(rmx_ctx* c, int64_t V, int k, int dtype, rmx_table** out) {
  CHECK_ARG(c && out && V > 0 && k >= 0, "rmx_table_create: bad args");
  CHECK_ARG(V < (int64_t(1) << 31), "rmx_table_create: rows must fit int32 (ParRecModel.scala:282 .toInt)");
  CHECK_ARG(dtype == RMX_DTYPE_F32 || dtype == RMX_DTYPE_BF16, "rmx_table_create: dtype must be F32 or BF16");
  RMX_HIP(hipSetDevice(c->device));
  auto* t = new rmx_table();
  t->ctx = c;
  t->V = V;
  t->k = k;
  t->dtype = dtype;
  const size_t es = dtype_size(dtype);
  if (hipMalloc(&t->w, es * V) != hipSuccess || (k > 0 && hipMalloc(&t->emb, es * V * k) != hipSuccess)) {
    if (t->w) (void)hipFree(t->w);
    delete t;
    set_error("rmx_table_create: out of device memory");
    return RMX_E_NOMEM;
  }
  *out = t;
  return RMX_OK;
}

extern "C" int rmx_table_create(rmx_ctx* c, int64_t V, int k, rmx_table** out) {
  return rmx_table_create_ex(c, V, k, RMX_DTYPE_F32, out);
}

// the [V][32] line copy of a k = 16 table (rmx_table::line; fp32 or bf16 elements), rebuilt from emb / w;
// knob "table_lines" 0 drops it (the forward then reads emb / w)
int rmx::table_refresh_lines(rmx_table& t) {
  const bool want = t.k == 16 && tuning_get("table_lines", 0) != 0;
  if (!want) {
    if (t.line) {
      RMX_HIP(hipStreamSynchronize(t.ctx->stream));
      (void)hipFree(t.line);
      t.line = nullptr;
    }
    return RMX_OK;
  }
  const size_t es = t.dtype == RMX_DTYPE_BF16 ? sizeof(bf16_t) : sizeof(float);
  if (!t.line && hipMalloc(&t.line, es * 32 * t.V) != hipSuccess) {
    t.line = nullptr;
    set_error("rmx_table: out of device memory for the line copy (set knob table_lines 0)");
    return RMX_E_NOMEM;
  }
  const int st = launch_pack_lines(t.ctx->stream, t.V, t.emb, t.w, t.line, t.dtype);
  if (st) return st;
  RMX_HIP(hipStreamSynchronize(t.ctx->stream));
  return RMX_OK;
}

extern "C" int rmx_table_refresh_lines(rmx_table* t) {
  CHECK_ARG(t, "rmx_table_refresh_lines: NULL table");
  RMX_HIP(hipSetDevice(t->ctx->device));
  return table_refresh_lines(*t);
}

extern "C" int rmx_table_destroy(rmx_table* t) {
  if (!t) return RMX_OK;
  (void)hipSetDevice(t->ctx->device);
  (void)hipStreamSynchronize(t->ctx->stream);
  if (t->w) (void)hipFree(t->w);
  if (t->emb) (void)hipFree(t->emb);
  if (t->line) (void)hipFree(t->line);
  delete t;
  return RMX_OK;
}

extern "C" int64_t rmx_table_rows(const rmx_table* t) { return t ? t->V : -1; }
extern "C" int rmx_table_dtype(const rmx_table* t) { return t ? t->dtype : -1; }
extern "C" int rmx_table_embedding_dim(const rmx_table* t) { return t ? t->k : -1; }

extern "C" int rmx_table_device_ptrs(const rmx_table* t, void** w, void** e) {
  CHECK_ARG(t, "rmx_table_device_ptrs: NULL");
  if (w) *w = t->w;
  if (e) *e = t->emb;
  return RMX_OK;
}

extern "C" int rmx_table_upload(rmx_table* t, const float* weights, const float* emb, int layout) {
  CHECK_ARG(t, "rmx_table_upload: NULL table");
  CHECK_ARG(layout == RMX_LAYOUT_K_MAJOR || layout == RMX_LAYOUT_ROW_MAJOR, "rmx_table_upload: bad layout");
  hipStream_t s = t->ctx->stream;
  RMX_HIP(hipSetDevice(t->ctx->device));
  const bool bf = t->dtype == RMX_DTYPE_BF16;
  // fp32 host arrays; a bf16 table stores them rounded to nearest even on the device
  const size_t need = (size_t)t->V * std::max(1, bf || layout == RMX_LAYOUT_K_MAJOR ? t->k : 0);
  float* tmp = nullptr;
  if (bf || (emb && layout == RMX_LAYOUT_K_MAJOR)) {
    if (hipMalloc(&tmp, sizeof(float) * std::max<size_t>(need, t->V)) != hipSuccess) {
      set_error("rmx_table_upload: out of device memory for the staging copy");
      return RMX_E_NOMEM;
    }
  }
  int st = RMX_OK;
  if (weights) {
    if (bf) {
      RMX_HIP(hipMemcpyAsync(tmp, weights, sizeof(float) * t->V, hipMemcpyHostToDevice, s));
      st = launch_convert_bf16(s, tmp, t->V, (bf16_t*)t->w);
      RMX_HIP(hipStreamSynchronize(s));
    } else {
      RMX_HIP(hipMemcpyAsync(t->w, weights, sizeof(float) * t->V, hipMemcpyHostToDevice, s));
    }
  }
  if (st == RMX_OK && emb && t->k > 0) {
    const size_t bytes = sizeof(float) * t->V * t->k;
    if (layout == RMX_LAYOUT_ROW_MAJOR && !bf) {
      RMX_HIP(hipMemcpyAsync(t->emb, emb, bytes, hipMemcpyHostToDevice, s));
    } else {
      RMX_HIP(hipMemcpyAsync(tmp, emb, bytes, hipMemcpyHostToDevice, s));
      st = layout == RMX_LAYOUT_ROW_MAJOR ? launch_convert_bf16(s, tmp, t->V * t->k, (bf16_t*)t->emb)
                                          : launch_transpose_kmajor(s, tmp, t->V, t->k, t->emb, t->dtype);
    }
  }
  RMX_HIP(hipStreamSynchronize(s));
  if (tmp) (void)hipFree(tmp);
  if (st == RMX_OK) st = table_refresh_lines(*t);
  return st;
}

extern "C" int rmx_table_fill_synthetic(rmx_table* t, uint64_t seed) {
  CHECK_ARG(t, "rmx_table_fill_synthetic: NULL table");
  RMX_HIP(hipSetDevice(t->ctx->device));
  const int st = launch_fill_table(t->ctx->stream, seed, t->V, t->k, t->w, t->emb, t->dtype);
  if (st != RMX_OK) return st;
  RMX_HIP(hipStreamSynchronize(t->ctx->stream));
  return table_refresh_lines(*t);
}

extern "C" int rmx_gen_ids(rmx_ctx* c, uint64_t seed, int64_t row0, int32_t B, int32_t F, int64_t V,
                           int32_t* d_ids, void* stream) {
  CHECK_ARG(c && d_ids && B >= 0 && F > 0 && V >= F, "rmx_gen_ids: bad args");
  RMX_HIP(hipSetDevice(c->device));
  return launch_gen_ids(stream ? (hipStream_t)stream : c->stream, seed, row0, B, F, V, d_ids);
}

// Test hook: every workgroup takes a whole CU's LDS (160 KiB) and fills it with `pattern`, so a kernel
// launched next that reads LDS it never wrote sees that pattern rather than a benign leftover.
__global__ __launch_bounds__(1024) void fill_lds_kernel(uint32_t pattern, int words) {
  extern __shared__ uint32_t fl_lds[];
  volatile uint32_t* l = fl_lds;  // (volatile: stores nothing reads back)
  for (int i = threadIdx.x; i < words; i += blockDim.x) l[i] = pattern;
}

extern "C" int rmx_debug_fill_lds(rmx_ctx* c, uint32_t pattern, void* stream) {
  CHECK_ARG(c, "rmx_debug_fill_lds: NULL context");
  RMX_HIP(hipSetDevice(c->device));
  int ncu = 256;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) ncu = 256;
  const int lds = 160 * 1024;  // gfx950: the whole LDS of a CU
  RMX_HIP(hipFuncSetAttribute((const void*)fill_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(fill_lds_kernel, dim3(4 * ncu), dim3(1024), (size_t)lds, stream ? (hipStream_t)stream : c->stream,
                     pattern, lds / 4);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

extern "C" int rmx_gen_ids_zipf(rmx_ctx* c, uint64_t seed, int64_t row0, int32_t B, int32_t F, int64_t V,
                                double exponent, int32_t* d_ids, void* stream) {
  CHECK_ARG(c && d_ids && B >= 0 && F > 0 && V >= F && exponent > 0.0 && exponent != 1.0,
            "rmx_gen_ids_zipf: bad args (exponent > 0, != 1)");
  RMX_HIP(hipSetDevice(c->device));
  return launch_gen_ids_zipf(stream ? (hipStream_t)stream : c->stream, seed, row0, B, F, V, exponent, d_ids);
}

extern "C" int rmx_gather(const rmx_table* t, int64_t n, const int32_t* d_ids, float* d_w, float* d_emb,
                          void* stream) {
  CHECK_ARG(t && d_ids && n >= 0, "rmx_gather: bad args");
  RMX_HIP(hipSetDevice(t->ctx->device));
  return launch_gather(stream ? (hipStream_t)stream : t->ctx->stream, n, d_ids, t->w, t->emb, t->dtype, t->k, d_w,
                       d_emb);
}

// ------------------------------------------------------------------ forward --
extern "C" int rmx_forward_ids(rmx_model* m, const rmx_table* t, int32_t B, const int32_t* d_ids,
                               float* d_out, void* stream) {
  CHECK_ARG(m && t && d_out && B >= 0, "rmx_forward_ids: bad args");
  CHECK_ARG(m->ctx, "rmx_forward_ids: host-only model (created without a context)");
  CHECK_ARG(d_ids || B == 0, "rmx_forward_ids: ids is NULL");
  if (!m->params_ready && m->mats_len > 0) {
    set_error("rmx_forward_ids: call rmx_model_set_mats first");
    return RMX_E_INVALID;
  }
  if (!m->beta_set) {
    set_error("rmx_forward_ids: call rmx_model_set_bias first");
    return RMX_E_INVALID;
  }
  if (m->type != RMX_MODEL_LR && t->k != m->k) {
    set_error("rmx_forward_ids: table embedding_dim " + std::to_string(t->k) + " != model " +
              std::to_string(m->k));
    return RMX_E_SHAPE;
  }
  if (m->type != RMX_MODEL_LR && t->dtype != m->precision) {
    set_error("rmx_forward_ids: table dtype differs from the model precision (rmx_model_set_precision)");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  ModelUse use(*m, s);
  if (use.st) return use.st;
  FwdInputs in;
  in.B = B;
  in.ids = d_ids;
  table_inputs(*t, *m, in);
  in.beta = m->beta;
  in.out = d_out;
  return model_forward(*m, s, in);
}

extern "C" int rmx_encoder_ids(rmx_model* m, const rmx_table* t, int32_t B, const int32_t* d_ids, float* d_y,
                               void* stream) {
  CHECK_ARG(m && t && d_ids && d_y && B >= 0 && m->ctx, "rmx_encoder_ids: bad args");
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  const int mode = m->type == RMX_MODEL_DEEPFM ? 1 : 0;
  // the table's [emb | w | pad] line copy when it has one (knob table_lines): one 128-B line per id
  FwdInputs in;
  table_inputs(*t, *m, in);
  return launch_encoder(s, mode, B, d_ids, in.table, in.wtab, t->dtype, m->F, t->k, d_y, nullptr, nullptr, in.ld,
                        in.wld);
}

// The params-map contract shared by RecModel.forward / backward (RecModel.scala:130-155):
// required keys per RecModelType, Reshape(B, F, k), matSizes, Scatter's index bound.
static int check_la(rmx_model* m, int32_t B, int64_t nnz, const int64_t* index, const float* bias,
                    const float* weights, const float* embedding, int32_t embedding_dim, const float* mats,
                    const int32_t* mat_sizes, int32_t n_sizes, bool* pregular, bool* psorted) {
  // params-map keys required by the model's RecModelType (NoSuchElementException in the reference)
  if (!bias) { set_error("key not found: bias"); return RMX_E_INVALID; }
  const bool needs_w = m->type != RMX_MODEL_DNN;
  const bool needs_emb = m->type != RMX_MODEL_LR;
  if (nnz > 0 && !index) { set_error("key not found: index"); return RMX_E_INVALID; }
  if (needs_w && nnz > 0 && !weights) { set_error("key not found: weights"); return RMX_E_INVALID; }
  if (needs_emb) {
    if (!embedding && nnz > 0) { set_error("key not found: embedding"); return RMX_E_INVALID; }
    if (m->mats_len > 0 && !mats) { set_error("key not found: mats"); return RMX_E_INVALID; }
    if (embedding_dim != m->k) {
      set_error("embedding_dim " + std::to_string(embedding_dim) + " != model embeddingDim " +
                std::to_string(m->k));
      return RMX_E_SHAPE;
    }
    if (nnz != (int64_t)B * m->F) {
      set_error("Reshape(" + std::to_string(B) + ", " + std::to_string(m->F) + ", " + std::to_string(m->k) +
                "): input has " + std::to_string(nnz * m->k) + " elements");
      return RMX_E_SHAPE;
    }
    if (mat_sizes) {
      if (n_sizes != (int)m->sizes.size() || !std::equal(m->sizes.begin(), m->sizes.end(), mat_sizes)) {
        set_error("matSizes differ from getMatsSize");
        return RMX_E_MATS;
      }
    }
  }
  // Scatter's require(index < batchSize) (bnn/Scatter.scala:29-30); .toInt at DeepFM.scala:28.
  bool regular = nnz == (int64_t)B * m->F && m->F > 0;
  bool sorted = true;
  for (int64_t n = 0; n < nnz; ++n) {
    const int32_t ix = (int32_t)index[n];
    if (ix < 0 || ix >= B) {
      set_error("index should smaller than " + std::to_string(B) + ", but got " + std::to_string(ix));
      return RMX_E_INDEX;
    }
    if (regular && ix != (int32_t)(n / m->F)) regular = false;
    if (n > 0 && ix < (int32_t)index[n - 1]) sorted = false;
  }
  *pregular = regular;
  *psorted = sorted;
  return RMX_OK;
}

extern "C" int rmx_forward(rmx_model* m, int32_t B, int64_t nnz, const int64_t* index, const int64_t* feats,
                           const float* bias, const float* weights, const float* embedding,
                           int32_t embedding_dim, const float* mats, const int32_t* mat_sizes,
                           int32_t n_sizes, const int64_t* fields, float* out) {
  (void)feats;
  (void)fields;  // no reference model reads "fields" 
  CHECK_ARG(m, "rmx_forward: model is NULL");
  CHECK_ARG(m->ctx, "rmx_forward: host-only model (created without a context)");
  CHECK_ARG(out || B == 0, "rmx_forward: out is NULL");
  CHECK_ARG(B >= 0 && nnz >= 0, "rmx_forward: negative batch_size / nnz");
  bool regular = false, sorted = false;
  int st = check_la(m, B, nnz, index, bias, weights, embedding, embedding_dim, mats, mat_sizes, n_sizes, &regular,
                    &sorted);
  if (st) return st;
  if (B == 0) return RMX_OK;
  RMX_HIP(hipSetDevice(m->ctx->device));
  ModelUse use(*m, m->ctx->stream);
  if (use.st) return use.st;
  return model_forward_host(*m, B, nnz, index, regular, sorted, bias[0], weights, embedding, mats, out);
}

// ------------------------------------------------------------- backward --

extern "C" int rmx_backward_ids(rmx_model* m, const rmx_table* t, int32_t B, const int32_t* d_ids,
                                const float* d_targets, float* d_g_bias, float* d_g_weights, float* d_g_embedding,
                                float* d_g_mats, float* d_loss, void* stream) {
  CHECK_ARG(m && t && B >= 0, "rmx_backward_ids: bad args");
  CHECK_ARG(m->ctx, "rmx_backward_ids: host-only model (created without a context)");
  CHECK_ARG((d_ids && d_targets) || B == 0, "rmx_backward_ids: ids / targets is NULL");
  if (!m->params_ready && m->mats_len > 0) {
    set_error("rmx_backward_ids: call rmx_model_set_mats first");
    return RMX_E_INVALID;
  }
  if (!m->beta_set) {
    set_error("rmx_backward_ids: call rmx_model_set_bias first");
    return RMX_E_INVALID;
  }
  if (m->type != RMX_MODEL_LR && t->k != m->k) {
    set_error("rmx_backward_ids: table embedding_dim differs from the model's");
    return RMX_E_SHAPE;
  }
  if (t->dtype != RMX_DTYPE_F32) {
    set_error("rmx_backward_ids: fp32 tables only");
    return RMX_E_INVALID;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : m->ctx->stream;
  ModelUse use(*m, s);
  if (use.st) return use.st;
  FwdInputs in;
  in.B = B;
  in.ids = d_ids;
  in.table = t->emb;
  in.wtab = t->w;
  in.dtype = t->dtype;
  in.beta = m->beta;
  TrainOutputs o;
  o.targets = d_targets;
  o.nnz = (int64_t)B * m->F;
  o.g_bias = d_g_bias;
  o.g_w = d_g_weights;
  o.g_emb = m->type == RMX_MODEL_LR ? nullptr : d_g_embedding;
  o.g_mats = d_g_mats;
  o.loss = d_loss;
  return model_train(*m, s, in, o);
}

extern "C" int rmx_backward(rmx_model* m, int32_t B, int64_t nnz, const int64_t* index, const int64_t* feats,
                            float* bias, float* weights, float* embedding, int32_t embedding_dim, float* mats,
                            const int32_t* mat_sizes, int32_t n_sizes, const int64_t* fields, const float* targets,
                            float* loss) {
  (void)feats;
  (void)fields;
  CHECK_ARG(m, "rmx_backward: model is NULL");
  CHECK_ARG(m->ctx, "rmx_backward: host-only model (created without a context)");
  CHECK_ARG(B >= 0 && nnz >= 0, "rmx_backward: negative batch_size / nnz");
  if (!targets && B > 0) { set_error("key not found: targets"); return RMX_E_INVALID; }
  bool regular = false, sorted = false;
  int st = check_la(m, B, nnz, index, bias, weights, embedding, embedding_dim, mats, mat_sizes, n_sizes, &regular,
                    &sorted);
  if (st) return st;
  if (B == 0) {
    if (loss) *loss = 0.f;
    return RMX_OK;
  }
  RMX_HIP(hipSetDevice(m->ctx->device));
  hipStream_t s = m->ctx->stream;
  ModelUse use(*m, s);
  if (use.st) return use.st;
  FwdInputs in;
  if ((st = model_stage_host(*m, B, nnz, index, regular, sorted, bias[0], weights, embedding, mats, &in))) return st;
  rmx_model::LaGrad* lb = &m->la_grad;
  const bool use_w = m->type != RMX_MODEL_DNN, use_e = m->type != RMX_MODEL_LR;
  if (nnz > lb->nnz || B > lb->B || m->mats_len > lb->ml) {
    RMX_HIP(hipDeviceSynchronize());
    for (void* p : {(void*)lb->gw, (void*)lb->ge, (void*)lb->gm, (void*)lb->gb, (void*)lb->tg, (void*)lb->idx})
      if (p) (void)hipFree(p);
    *lb = rmx_model::LaGrad{};
    const int64_t n1 = std::max<int64_t>(nnz, 1);
    if (hipMalloc(&lb->gw, sizeof(float) * n1) != hipSuccess ||
        hipMalloc(&lb->ge, sizeof(float) * n1 * std::max(m->k, 1)) != hipSuccess ||
        hipMalloc(&lb->gm, sizeof(float) * std::max<int64_t>(m->mats_len, 1)) != hipSuccess ||
        hipMalloc(&lb->gb, sizeof(float) * 2) != hipSuccess || hipMalloc(&lb->tg, sizeof(float) * B) != hipSuccess ||
        hipMalloc(&lb->idx, sizeof(int32_t) * n1) != hipSuccess) {
      set_error("rmx_backward: out of device memory");
      return RMX_E_NOMEM;
    }
    lb->nnz = nnz;
    lb->B = B;
    lb->ml = m->mats_len;
  }
  RMX_HIP(hipMemcpyAsync(lb->tg, targets, sizeof(float) * B, hipMemcpyHostToDevice, s));
  std::vector<int32_t> idx32;
  if (use_w && !regular) {
    idx32.resize(nnz);
    for (int64_t n = 0; n < nnz; ++n) idx32[n] = (int32_t)index[n];
    RMX_HIP(hipMemcpyAsync(lb->idx, idx32.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice, s));
  }
  TrainOutputs o;
  o.targets = lb->tg;
  o.index = (use_w && !regular) ? lb->idx : nullptr;
  o.nnz = nnz;
  o.g_bias = lb->gb;
  o.g_w = use_w ? lb->gw : nullptr;
  o.g_emb = use_e ? lb->ge : nullptr;
  o.g_mats = m->mats_len > 0 ? lb->gm : nullptr;
  o.loss = lb->gb + 1;
  if ((st = model_train(*m, s, in, o))) return st;
  // RecModel.backward's write-back: the caller's arrays now hold the gradients (GradUtil.scala)
  float hb[2];
  RMX_HIP(hipMemcpyAsync(hb, lb->gb, sizeof(float) * 2, hipMemcpyDeviceToHost, s));
  if (use_w && nnz > 0) RMX_HIP(hipMemcpyAsync(weights, lb->gw, sizeof(float) * nnz, hipMemcpyDeviceToHost, s));
  if (use_e && nnz > 0)
    RMX_HIP(hipMemcpyAsync(embedding, lb->ge, sizeof(float) * nnz * m->k, hipMemcpyDeviceToHost, s));
  if (m->mats_len > 0) RMX_HIP(hipMemcpyAsync(mats, lb->gm, sizeof(float) * m->mats_len, hipMemcpyDeviceToHost, s));
  RMX_HIP(hipStreamSynchronize(s));
  bias[0] = hb[0];
  if (loss) *loss = hb[1];
  return RMX_OK;
}
