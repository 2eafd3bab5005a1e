// models.hip -- per-model layer plans, parameter packing and forward sequences.
//
// Layer plans restate the mats offset walk of each reference model (LayerUtil.buildLinear at
// running offsets, util/LayerUtil.scala:7-40):
//   DeepFM / DNN  model/encoder/HigherOrderEncoder.scala:48-58
//   xDeepFM       model/xdeepfm/CINEncoder.scala:123-176
//   DCN           model/dcn/CrossEncoder.scala:134-185
//   PNN           model/pnn/ProductEncoder.scala:72-108 + PNN.scala:78 (tail tower, start = end offset)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "rmx_models.hpp"

namespace rmx {

namespace {

void push(std::vector<int32_t>& v, int a, int b) {
  v.push_back(a);
  v.push_back(b);
}

// getMatsSize of each model (see oracle/rmx_oracle.c for the per-model file:line).
std::vector<int32_t> mats_sizes(const rmx_model& m) {
  std::vector<int32_t> s;
  const int F = m.F, k = m.k, D = F * k;
  switch (m.type) {
    case RMX_MODEL_LR:
      break;
    case RMX_MODEL_DEEPFM:
    case RMX_MODEL_DNN: {
      int prev = D;
      for (size_t i = 0; i <= m.fc.size(); ++i) {
        const int cur = i < m.fc.size() ? m.fc[i] : 1;
        push(s, prev, cur);
        push(s, cur, 1);
        prev = cur;
      }
      break;
    }
    case RMX_MODEL_XDEEPFM: {
      int prev = D;
      for (int d : m.fc) {
        push(s, prev, d);
        push(s, d, 1);
        prev = d;
      }
      int hp = F, sum = 0;
      for (int h : m.cin) {
        push(s, F * hp, h);
        push(s, h, 1);
        hp = h;
        sum += h;
      }
      push(s, sum + m.fc.back(), 1);
      break;
    }
    case RMX_MODEL_DCN: {
      for (int i = 0; i < m.cross_depth; ++i) push(s, D, 1);
      for (int i = 0; i < m.cross_depth; ++i) push(s, 1, 1);
      int prev = D;
      for (int d : m.fc) {
        push(s, prev, d);
        push(s, d, 1);
        prev = d;
      }
      push(s, D + m.fc.back(), 1);
      break;
    }
    case RMX_MODEL_PNN: {
      const int P = F * (F - 1) / 2;
      push(s, D, m.fc[0]);
      push(s, P, m.fc[0]);
      push(s, 1, 1);
      int prev = m.fc[0];
      for (size_t i = 1; i <= m.fc.size(); ++i) {
        const int cur = i < m.fc.size() ? m.fc[i] : 1;
        push(s, prev, cur);
        push(s, cur, 1);
        prev = cur;
      }
      break;
    }
  }
  return s;
}

float bf16_round_host(float f) {  // round to nearest even, finite values
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  u &= 0xFFFF0000u;
  std::memcpy(&f, &u, 4);
  return f;
}

uint64_t splitmix64_h(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

float unif_h(uint64_t h, float a) {
  const float scale = a * (1.0f / 8388608.0f);
  return (float)((int32_t)(h >> 40) - 8388608) * scale;
}

DenseLayer make_layer(int K, int N, int64_t w_off, int64_t b_off) {
  DenseLayer L;
  L.K = K;
  L.N = N;
  L.Kpad = round_up(K, kChunk);
  L.Npad = tower_npad_for(N);
  L.w_off = w_off;
  L.b_off = b_off;
  return L;
}

int dev_alloc(float** p, size_t n) {
  if (hipMalloc(p, sizeof(float) * (n ? n : 1)) != hipSuccess) {
    set_error("out of device memory (" + std::to_string(n * 4) + " bytes)");
    return RMX_E_NOMEM;
  }
  return RMX_OK;
}

int dev_alloc_bf16(bf16_t** p, int64_t n) {
  if (hipMalloc(p, sizeof(bf16_t) * (n > 0 ? n : 1)) != hipSuccess) {
    set_error("out of device memory (" + std::to_string(n * 2) + " bytes)");
    return RMX_E_NOMEM;
  }
  return RMX_OK;
}

template <class T>
void dev_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// W^T planes for the backward's dX on the split GEMM (single-block fp32 layers whose input width
// pads to a multiple of 208 with at most one extra 16-wide tile, e.g. 400 -> 416, 624; the dX buffer's
// row stride must also hold NTpad, checked at launch: dx_s3_usable)
int alloc_wt(DenseLayer& L) {
  dev_free(L.WT);
  dev_free(L.WT3);
  L.KTpad = L.NTpad = 0;
  if (L.K1 >= 0 || L.N1 >= 0 || round_up(L.K, 208) - round_up(L.K, kChunk) > kChunk) return RMX_OK;
  L.KTpad = round_up(L.N, kChunk);
  L.NTpad = round_up(L.K, 208);
  int st = dev_alloc(&L.WT, (size_t)L.KTpad * L.NTpad);
  if (!st) st = dev_alloc_bf16(&L.WT3, split3_elems(L.KTpad / kChunk, L.NTpad));
  return st;
}

// the GEMM gathers 16-B slots straight from table rows: k must be a multiple of 4 fp32 / 8 bf16
bool needs_gather_x(const rmx_model& m) { return m.k % (m.precision == kBF16 ? 8 : 4) != 0; }

// row stride (elements) of the materialised layer-1 input xbuf (PNN [x | ip], generic-k x): Kpad
// rounded up to whole 128-B lines, so no row of the GEMM's A operand straddles a line boundary
// (PNN bf16: 1,376 -> 1,408 elements; fp32 rows of 1,376 are already 43 lines)
int xbuf_ld_max(const rmx_model& m) { return round_up(m.layers[0].Kpad, m.precision == kBF16 ? 64 : 32); }
int xbuf_ld(const rmx_model& m) { return tuning_get("x_line_pad", 1) ? xbuf_ld_max(m) : m.layers[0].Kpad; }

}  // namespace

int model_build(rmx_model& m) {
  const int t = m.type;
  if (t != RMX_MODEL_LR) {
    if (m.F <= 0 || m.k <= 0) {
      set_error("nFields and embeddingDim must be positive");
      return RMX_E_INVALID;
    }
    // "".split(",").map(_.toInt) throws in the reference (example/*LocalExample.scala:21)
    if (m.fc.empty()) {
      set_error("fcDims must not be empty");
      return RMX_E_INVALID;
    }
    for (int d : m.fc)
      if (d <= 0) {
        set_error("fcDims must be positive");
        return RMX_E_INVALID;
      }
  }
  if (t == RMX_MODEL_XDEEPFM) {
    if (m.cin.empty()) {
      set_error("cinDims must not be empty");
      return RMX_E_INVALID;
    }
    if (m.k != 16) {
      set_error("xDeepFM CIN kernel supports embeddingDim 16 only");
      return RMX_E_INVALID;
    }
    for (int h : m.cin)
      if (h <= 0 || h > 256) {
        set_error("cinDims must be in [1, 256]");
        return RMX_E_INVALID;
      }
  }
  if (t == RMX_MODEL_DCN) {
    if (m.cross_depth <= 0) {  // (0 until 0).map(...).reduce throws (DCN.scala:17-19)
      set_error("crossDepth must be positive");
      return RMX_E_INVALID;
    }
    if (m.F * m.k > 1024) {
      set_error("DCN cross kernel supports nFields*embeddingDim <= 1024");
      return RMX_E_INVALID;
    }
  }
  if (t == RMX_MODEL_PNN && m.F < 2) {
    set_error("PNN needs at least two fields");
    return RMX_E_INVALID;
  }
  m.sizes = mats_sizes(m);
  m.mats_len = 0;
  for (size_t i = 0; i < m.sizes.size(); i += 2) m.mats_len += (int64_t)m.sizes[i] * m.sizes[i + 1];

  const int D = m.F * m.k;
  int64_t off = 0;
  switch (t) {
    case RMX_MODEL_LR:
      break;
    case RMX_MODEL_DEEPFM:
    case RMX_MODEL_DNN: {
      int prev = D;
      for (int d : m.fc) {
        m.layers.push_back(make_layer(prev, d, off, off + (int64_t)prev * d));
        off += (int64_t)prev * d + d;
        prev = d;
      }
      m.wo_off = off;
      m.bo_off = off + prev;
      m.has_bo = true;
      break;
    }
    case RMX_MODEL_XDEEPFM: {
      int prev = D;
      for (int d : m.fc) {
        m.layers.push_back(make_layer(prev, d, off, off + (int64_t)prev * d));
        off += (int64_t)prev * d + d;
        prev = d;
      }
      int hp = m.F, sum = 0, hp_pad = round_up(m.F, 16);
      for (int h : m.cin) {
        CinLayer c;
        c.Hp = hp;
        c.Hp_pad = hp_pad;  // = the previous layer's Npad (its maps' row stride)
        c.H = h;
        c.Npad = cin_npad_for(h);
        hp_pad = c.Npad;
        c.w_off = off;
        c.b_off = off + (int64_t)m.F * hp * h;
        off += (int64_t)m.F * hp * h + h;
        hp = h;
        sum += h;
        m.cin_layers.push_back(c);
      }
      m.wo_cin_off = off;
      int base = 0;
      for (auto& c : m.cin_layers) {
        c.wo_off = off + base;
        base += c.H;
      }
      m.wo_off = off + sum;  // the DNN slice of the output Linear (no bias)
      m.has_bo = false;
      break;
    }
    case RMX_MODEL_DCN: {
      m.cross_w_off = 0;
      m.cross_b_off = (int64_t)m.cross_depth * D;
      off = m.cross_b_off + m.cross_depth;
      // fcDims >= 2: the cross dots x0.w_l and x0.W_out[0:D] ride along tower layer 1 (same A = x0)
      // as L + 1 raw extra columns, and the cross stack collapses to a per-row closed form
      m.dcn_fused = m.fc.size() >= 2 && m.cross_depth <= kMaxFusedCross;
      int prev = D;
      for (int d : m.fc) {
        const bool first = m.layers.empty();
        DenseLayer L = make_layer(prev, first && m.dcn_fused ? d + m.cross_depth + 1 : d, off,
                                  off + (int64_t)prev * d);
        if (first && m.dcn_fused) {
          L.N1 = d;
          L.nx = m.cross_depth;
          L.w_off_x = m.cross_w_off;
        }
        m.layers.push_back(L);
        off += (int64_t)prev * d + d;
        prev = d;
      }
      m.wo_x_off = off;
      m.wo_off = off + D;
      if (m.dcn_fused) m.layers[0].w_off_o = m.wo_x_off;
      m.has_bo = false;
      break;
    }
    case RMX_MODEL_PNN: {
      const int P = m.F * (m.F - 1) / 2, D1 = m.fc[0];
      DenseLayer L0 = make_layer(D + P, D1, 0, (int64_t)D * D1 + (int64_t)P * D1);
      L0.K1 = D;
      L0.w_off2 = (int64_t)D * D1;
      L0.bias_mode = 2;
      m.layers.push_back(L0);
      off = (int64_t)D * D1 + (int64_t)P * D1 + 1;
      int prev = D1;
      for (size_t i = 1; i < m.fc.size(); ++i) {
        const int d = m.fc[i];
        m.layers.push_back(make_layer(prev, d, off, off + (int64_t)prev * d));
        off += (int64_t)prev * d + d;
        prev = d;
      }
      m.wo_off = off;
      m.bo_off = off + prev;
      m.has_bo = true;
      break;
    }
  }
  if (t != RMX_MODEL_LR && off + (m.has_bo ? m.layers.back().N + 1 : 0) != m.mats_len &&
      t != RMX_MODEL_XDEEPFM && t != RMX_MODEL_DCN) {
    set_error("internal: mats layout mismatch");
    return RMX_E_INVALID;
  }

  if (!m.ctx) return RMX_OK;  // host-only model: metadata only
  // device parameter buffers
  RMX_HIP(hipSetDevice(m.ctx->device));
  int st = RMX_OK;
  if (m.mats_len > 0 && (st = dev_alloc(&m.mats_dev, m.mats_len))) return st;
  for (auto& L : m.layers) {
    if ((st = dev_alloc(&L.W, (size_t)L.Kpad * L.Npad))) return st;
    if ((st = dev_alloc_bf16(&L.W3, split3_elems(L.Kpad / kChunk, L.Npad)))) return st;
    if ((st = dev_alloc(&L.b, L.Npad))) return st;
    if ((st = alloc_wt(L))) return st;
  }
  if (!m.layers.empty()) {
    if ((st = dev_alloc(&m.wo, m.layers.back().Npad))) return st;
  }
  for (auto& c : m.cin_layers) {
    if ((st = dev_alloc(&c.W, (size_t)c.Hp_pad * m.F * c.Npad))) return st;
    if ((st = dev_alloc_bf16(&c.W3, split3_elems(c.Hp_pad / kChunk * m.F, c.Npad)))) return st;
    {  // the split kernel's K order (k_gemm.hip cin_chunk_map): at most Hp_pad / 16 * F chunks
      c.tri = &c == &m.cin_layers.front() ? 1 : 0;
      const std::vector<int> map = cin_chunk_map(m.F, c.Hp, c.tri != 0);
      c.ncm = (int)map.size();
      if (hipMalloc(&c.cmap, sizeof(int) * std::max<size_t>(map.size(), 1)) != hipSuccess) {
        set_error("out of device memory (CIN chunk map)");
        return RMX_E_NOMEM;
      }
      RMX_HIP(hipMemcpy(c.cmap, map.data(), sizeof(int) * map.size(), hipMemcpyHostToDevice));
      if ((st = dev_alloc(&c.Wm, (size_t)c.ncm * c.Npad * 16))) return st;
    }
    c.KTpad = round_up(c.H, kChunk);
    c.NTpad = round_up(m.F * c.Hp, 208);
    if ((st = dev_alloc(&c.WT, (size_t)c.KTpad * c.NTpad))) return st;
    if ((st = dev_alloc_bf16(&c.WT3, split3_elems(c.KTpad / kChunk, c.NTpad)))) return st;
    if ((st = dev_alloc(&c.b, c.Npad))) return st;
    if ((st = dev_alloc(&c.wo, c.Npad))) return st;
  }
  if (t == RMX_MODEL_DCN) {
    if ((st = dev_alloc(&m.cross_w, (size_t)m.cross_depth * D))) return st;
    if ((st = dev_alloc(&m.cross_b, m.cross_depth))) return st;
    if ((st = dev_alloc(&m.wo_x, D))) return st;
  }
  if (t == RMX_MODEL_PNN) {
    // pairs (i < j) lexicographic: ProductEncoder.calcIndices (ProductEncoder.scala:110-120)
    std::vector<int32_t> pr;
    for (int i = 0; i < m.F; ++i)
      for (int j = i + 1; j < m.F; ++j) {
        pr.push_back(i);
        pr.push_back(j);
      }
    if (hipMalloc(&m.pairs, sizeof(int32_t) * pr.size()) != hipSuccess) {
      set_error("out of device memory");
      return RMX_E_NOMEM;
    }
    RMX_HIP(hipMemcpy(m.pairs, pr.data(), sizeof(int32_t) * pr.size(), hipMemcpyHostToDevice));
  }
  return RMX_OK;
}

// Synthetic parameters: Xavier-uniform +-sqrt(6/(in+out)) for every Linear
// weight, U(-0.01, 0.01) for biases, value i of a segment from splitmix64(seed ^ (offset + i)).
// Which getMatsSize pairs are biases follows the LayerUtil calls of each model.
void model_init_mats(const rmx_model& m, uint64_t seed, float* mats) {
  int64_t off = 0;
  const int npairs = (int)m.sizes.size() / 2;
  for (int pair = 0; pair < npairs; ++pair) {
    const int a = m.sizes[2 * pair], b = m.sizes[2 * pair + 1];
    const int64_t len = (int64_t)a * b;
    bool is_bias = false;
    switch (m.type) {
      case RMX_MODEL_DEEPFM:
      case RMX_MODEL_DNN:
        is_bias = pair & 1;
        break;
      case RMX_MODEL_XDEEPFM: {
        const int nfc = 2 * (int)m.fc.size(), ncin = 2 * (int)m.cin.size();
        is_bias = pair < nfc + ncin ? ((pair < nfc ? pair : pair - nfc) & 1) : false;
        break;
      }
      case RMX_MODEL_DCN: {
        const int L = m.cross_depth, nfc = 2 * (int)m.fc.size();
        if (pair < L) is_bias = false;
        else if (pair < 2 * L) is_bias = true;
        else if (pair < 2 * L + nfc) is_bias = (pair - 2 * L) & 1;
        break;
      }
      case RMX_MODEL_PNN:
        is_bias = pair < 2 ? false : (pair == 2 ? true : ((pair - 3) & 1));
        break;
      default:
        break;
    }
    const float amp = is_bias ? 0.01f : sqrtf(6.0f / (float)(a + b));
    for (int64_t i = 0; i < len; ++i) mats[off + i] = unif_h(splitmix64_h(seed ^ (uint64_t)(off + i)), amp);
    off += len;
  }
}

void model_release(rmx_model& m) {
  train_release(m);
  for (void* p : {(void*)m.la_grad.gw, (void*)m.la_grad.ge, (void*)m.la_grad.gm, (void*)m.la_grad.gb,
                  (void*)m.la_grad.tg, (void*)m.la_grad.idx})
    if (p) (void)hipFree(p);
  m.la_grad = rmx_model::LaGrad{};
  if (!m.ctx) return;
  (void)hipSetDevice(m.ctx->device);
  (void)hipDeviceSynchronize();  // the last calls may have run on any stream
  if (m.ws_fence) (void)hipEventDestroy(m.ws_fence);
  m.ws_fence = nullptr;
  dev_free(m.mats_dev);
  for (auto& L : m.layers) {
    dev_free(L.W);
    dev_free(L.W16);
    dev_free(L.W3);
    dev_free(L.WT);
    dev_free(L.WT3);
    dev_free(L.b);
  }
  dev_free(m.wo);
  for (auto& c : m.cin_layers) {
    dev_free(c.W);
    dev_free(c.W3);
    dev_free(c.Wm);
    dev_free(c.cmap);
    dev_free(c.WT);
    dev_free(c.WT3);
    dev_free(c.b);
    dev_free(c.wo);
  }
  dev_free(m.cross_w);
  dev_free(m.cross_b);
  dev_free(m.wo_x);
  dev_free(m.pairs);
  dev_free(m.h[0]);
  dev_free(m.h[1]);
  dev_free(m.y12);
  dev_free(m.pre2);
  dev_free(m.xcol);
  dev_free(m.xbuf);
  dev_free(m.ubuf[0]);
  dev_free(m.ubuf[1]);
  dev_free(m.rowdot);
  dev_free(m.opart);
  dev_free(m.la_E);
  dev_free(m.la_w);
  dev_free(m.la_E16);
  dev_free(m.la_w16);
  dev_free(m.la_rowptr);
  dev_free(m.la_out);
  for (auto& p : m.pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : m.ev_pool) (void)hipEventDestroy(e);
}

__global__ void copy_slice_kernel(const float* __restrict__ src, int n, int npad, float* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < npad) dst[i] = i < n ? src[i] : 0.f;
}

static int copy_slice(hipStream_t s, const float* src, int n, int npad, float* dst) {
  if (npad <= 0) return RMX_OK;
  hipLaunchKernelGGL(copy_slice_kernel, dim3((npad + 255) / 256), dim3(256), 0, s, src, n, npad, dst);
  RMX_HIP(hipGetLastError());
  return RMX_OK;
}

// Switch the parameter storage of the GEMM layers between fp32 and bf16 (before set_mats).
int model_set_precision(rmx_model& m, int dtype) {
  RMX_HIP(hipSetDevice(m.ctx->device));
  RMX_HIP(hipStreamSynchronize(m.ctx->stream));
  for (auto& L : m.layers) {
    dev_free(L.W);
    dev_free(L.W16);
    dev_free(L.W3);
    dev_free(L.WT);
    dev_free(L.WT3);
    L.Kpad = round_up(L.K, dtype == kBF16 ? 32 : kChunk);
    if (dtype == kBF16) {
      if (hipMalloc(&L.W16, sizeof(bf16_t) * (size_t)L.Kpad * L.Npad) != hipSuccess) {
        set_error("out of device memory");
        return RMX_E_NOMEM;
      }
    } else {
      int st = dev_alloc(&L.W, (size_t)L.Kpad * L.Npad);
      if (!st) st = dev_alloc_bf16(&L.W3, split3_elems(L.Kpad / kChunk, L.Npad));
      if (!st) st = alloc_wt(L);
      if (st) return st;
    }
  }
  m.precision = dtype;
  m.params_ready = false;
  // workspaces depend on Kpad (PNN [x | ip] rows): rebuild on the next call
  RMX_HIP(hipStreamSynchronize(m.ctx->stream));
  dev_free(m.xbuf);
  m.ws_B = 0;
  return RMX_OK;
}

// Upload mats and pack every layer on the device (the reference rebuilds its BigDL modules
// from mats on every call: LayerUtil.scala:13-19; here it is one H2D copy + pack kernels).
int model_load_mats(rmx_model& m, const float* host_mats, bool sync) {
  hipStream_t s = m.ctx->stream;
  RMX_HIP(hipSetDevice(m.ctx->device));
  if (m.mats_len > 0)
    RMX_HIP(hipMemcpyAsync(m.mats_dev, host_mats, sizeof(float) * m.mats_len, hipMemcpyHostToDevice, s));
  int st;
  for (auto& L : m.layers) {
    if ((st = launch_pack_linear(s, m.mats_dev, L))) return st;
    if (L.W3 && (st = launch_pack_split3(s, L.W, L.Kpad / kChunk, L.Npad, L.W3))) return st;
    if (L.WT && (st = launch_pack_linear_t(s, m.mats_dev, L))) return st;
  }
  if (!m.layers.empty()) {
    const auto& last = m.layers.back();
    if ((st = copy_slice(s, m.mats_dev + m.wo_off, last.N, last.Npad, m.wo))) return st;
    m.bo = m.has_bo ? host_mats[m.bo_off] : 0.f;
  }
  for (auto& c : m.cin_layers) {
    if ((st = launch_pack_cin(s, m.mats_dev, m.F, c))) return st;
    // knob "cin_map" (default 1): the split planes in the chunk-map order (layer 1 folded to h <= f,
    // paired fields on a half-live h-chunk); 0: the plain hc * F + f order of c.W
    c.map_on = c.W3 && c.cmap && tuning_get("cin_map", 1) != 0 ? 1 : 0;
    if (c.map_on && (st = launch_pack_cin_map(s, m.mats_dev, m.F, c))) return st;
    if (c.W3 && !c.map_on && (st = launch_pack_split3(s, c.W, c.Hp_pad / kChunk * m.F, c.Npad, c.W3))) return st;
    if (c.WT3 && (st = launch_pack_cin_t(s, m.mats_dev, m.F, c))) return st;
    if ((st = copy_slice(s, m.mats_dev + c.b_off, c.H, c.Npad, c.b))) return st;
    if ((st = copy_slice(s, m.mats_dev + c.wo_off, c.H, c.Npad, c.wo))) return st;
  }
  if (m.type == RMX_MODEL_DCN) {
    const int D = m.F * m.k;
    if (m.cross_depth <= kMaxFusedCross) {
      // closed-form scalars (the fused forward and the backward); the extra GEMM columns use the
      // packed (bf16-rounded for bf16 models) vectors, so the sums are taken over the same values
      auto rv = [&](float v) { return m.precision == kBF16 ? bf16_round_host(v) : v; };
      for (int l = 0; l < m.cross_depth; ++l) {
        double ws = 0.0;
        for (int d = 0; d < D; ++d) ws += rv(host_mats[m.cross_w_off + (int64_t)l * D + d]);
        m.cross_scalars.wsum[l] = (float)ws;
        m.cross_scalars.beta[l] = host_mats[m.cross_b_off + l];
      }
      double wo = 0.0;
      for (int d = 0; d < D; ++d) wo += rv(host_mats[m.wo_x_off + d]);
      m.cross_scalars.wo_sum = (float)wo;
    }
    RMX_HIP(hipMemcpyAsync(m.cross_w, m.mats_dev + m.cross_w_off, sizeof(float) * m.cross_depth * D,
                           hipMemcpyDeviceToDevice, s));
    RMX_HIP(hipMemcpyAsync(m.cross_b, m.mats_dev + m.cross_b_off, sizeof(float) * m.cross_depth,
                           hipMemcpyDeviceToDevice, s));
    RMX_HIP(hipMemcpyAsync(m.wo_x, m.mats_dev + m.wo_x_off, sizeof(float) * D, hipMemcpyDeviceToDevice, s));
  }
  if (sync) RMX_HIP(hipStreamSynchronize(s));
  m.params_ready = true;
  return RMX_OK;
}

namespace {

int ensure_ws(rmx_model& m, int B) {
  if (B <= m.ws_B) return RMX_OK;
  RMX_HIP(hipDeviceSynchronize());  // earlier calls on any stream may still read the old buffers
  dev_free(m.h[0]);
  dev_free(m.h[1]);
  dev_free(m.y12);
  dev_free(m.pre2);
  dev_free(m.xcol);
  dev_free(m.xbuf);
  dev_free(m.ubuf[0]);
  dev_free(m.ubuf[1]);
  dev_free(m.rowdot);
  dev_free(m.opart);
  int st;
  int maxN = 16;
  for (auto& L : m.layers) maxN = std::max(maxN, L.Npad);
  if (!m.layers.empty()) {
    if ((st = dev_alloc(&m.h[0], (size_t)B * maxN))) return st;
    if ((st = dev_alloc(&m.h[1], (size_t)B * maxN))) return st;
    // partial logits of an output layer run in column slices (k_gemm_s3.hip)
    // (up to Npad / 16 slices: 208-column slices, or the 32-column blocks of small batches, s3_cols)
    if ((st = dev_alloc(&m.opart, (size_t)B * (m.layers.back().Npad / 16 + 1)))) return st;
  }
  if ((st = dev_alloc(&m.y12, B))) return st;
  if ((st = dev_alloc(&m.pre2, B))) return st;
  if (m.dcn_fused && (st = dev_alloc(&m.xcol, (size_t)B * (m.cross_depth + 1)))) return st;
  if (m.type == RMX_MODEL_PNN || (m.type != RMX_MODEL_LR && needs_gather_x(m)) ||
      (m.type == RMX_MODEL_DEEPFM && B <= tuning_get("s3_cols", kS3ColsMaxB))) {
    if ((st = dev_alloc(&m.xbuf, (size_t)B * xbuf_ld_max(m)))) return st;
  }
  if (!m.cin_layers.empty()) {
    int maxH = 16;
    for (auto& c : m.cin_layers) maxH = std::max(maxH, c.Npad);
    if ((st = dev_alloc(&m.ubuf[0], (size_t)B * m.k * maxH))) return st;
    if ((st = dev_alloc(&m.ubuf[1], (size_t)B * m.k * maxH))) return st;
    if ((st = dev_alloc(&m.rowdot, (size_t)B * m.k))) return st;
  }
  m.ws_B = B;
  return RMX_OK;
}

// --- stage timing -----------------------------------------------------------

}  // namespace

int model_ensure_ws(rmx_model& m, int B) { return ensure_ws(m, B); }

static hipEvent_t take_event(rmx_model& m) {
  if (!m.ev_pool.empty()) {
    hipEvent_t e = m.ev_pool.back();
    m.ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}

StageTimer::StageTimer(rmx_model& mm, hipStream_t ss, const char* name) : m(mm), s(ss) {
  if (!m.timing) return;
  auto it = std::find(m.stage_names.begin(), m.stage_names.end(), std::string(name));
  if (it == m.stage_names.end()) {
    m.stage_names.push_back(name);
    m.stage_ms.push_back(0.f);
    idx = (int)m.stage_names.size() - 1;
  } else {
    idx = (int)(it - m.stage_names.begin());
  }
  a = take_event(m);
  (void)hipEventRecord(a, s);
}

StageTimer::~StageTimer() {
  if (!m.timing) return;
  hipEvent_t b = take_event(m);
  (void)hipEventRecord(b, s);
  m.pending.push_back({idx, a, b});
}

int model_collect_timing(rmx_model& m) {
  for (auto& p : m.pending) {
    RMX_HIP(hipEventSynchronize(p.b));
    float ms = 0.f;
    RMX_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    m.stage_ms[p.stage] += ms;
    m.ev_pool.push_back(p.a);
    m.ev_pool.push_back(p.b);
  }
  m.pending.clear();
  return RMX_OK;
}

// the models whose every table access in the forward takes a row / weight stride: LR, DeepFM / DNN (encoder,
// gathered layer 1), and DCN when its cross stack rides layer 1 (dcn_fused: the gathered layer 1 and the
// first-order kernel read the table, never cross16_kernel)
bool model_reads_lines(const rmx_model& m) {
  return m.type == RMX_MODEL_LR ||
         ((m.type == RMX_MODEL_DEEPFM || m.type == RMX_MODEL_DNN || (m.type == RMX_MODEL_DCN && m.dcn_fused)) &&
          m.k == 16 && !needs_gather_x(m));
}

void table_inputs(const rmx_table& t, const rmx_model& m, FwdInputs& in) {
  in.dtype = t.dtype;
  if (t.line && model_reads_lines(m)) {
    in.table = t.line;
    in.wtab = t.dtype == kBF16 ? (const void*)(reinterpret_cast<const bf16_t*>(t.line) + 16) : (const void*)(t.line + 16);
    in.ld = in.wld = 32;
  } else {
    in.table = t.emb;
    in.wtab = t.w;
    in.ld = in.wld = 0;
  }
}

// The per-model kernel sequence.  in.ids == nullptr means implicit ids (L-A gathered rows).
int model_forward(rmx_model& m, hipStream_t s, const FwdInputs& in) {
  const int B = in.B;
  if (B == 0) return RMX_OK;
  int st = ensure_ws(m, B);
  if (st) return st;
  if (m.timing) ++m.timed_calls;
  const int F = m.F, k = m.k;

  // strided ([emb | w | pad] line) tables reach only kernels that take a row stride: the encoder and
  // the gathered tower layer 1 (DeepFM / DNN / LR)
  const bool strided = (in.ld > 0 && in.ld != k) || in.wld > 1;
  if (strided && !model_reads_lines(m)) {
    set_error("forward: a strided (line-row) table needs LR, or a DeepFM / DNN / DCN (cross fused) model with k = 16");
    return RMX_E_INVALID;
  }
  if (m.type == RMX_MODEL_LR) {
    StageTimer t(m, s, "first_order_sigmoid");
    if (in.y1) return launch_sigmoid_out(s, B, in.y1, in.beta, in.out);
    return launch_encoder(s, 2, B, in.ids, nullptr, in.wtab, in.dtype, F, 0, nullptr, &in.beta, in.out, in.ld, in.wld);
  }

  // DeepFM fp32 at a small launch batch, column-split (round 6, knob "s3_cols" = the largest B that takes it):
  // the encoder writes the gathered rows x (and y1 + y2), then each layer runs on 128-row x 32-column blocks
  // that stream 1/13 of its split planes (k_gemm_s3.hip p.cols32), the output layer writing 13 partial logits
  // that out_finish_kernel sums in order with the head (layer 1 gathering its rows from the table instead of
  // the encoder's x measured slower: 0.031 vs 0.013 + 0.017 ms at B = 1,024, profiles/r06/ab_cols32_gather.txt).
  // Auto choice only: s3_small 0 (the per-layer paths) and 2 (the whole-tower kernel, below) both bypass it
  if (m.type == RMX_MODEL_DEEPFM && in.ids && !in.y1 && in.dtype == kF32 && !needs_gather_x(m) && k == 16 &&
      B <= tuning_get("s3_cols", kS3ColsMaxB) && tuning_get("s3_small", 1) == 1 && m.xbuf && m.layers.size() >= 2 &&
      m.layers[0].W3 && f32_split_enabled() && m.layers[0].Kpad == F * k) {
    {
      StageTimer t(m, s, "encoder_fm_x");
      if ((st = launch_encoder(s, 1, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr, nullptr, in.ld,
                               in.wld, m.xbuf)))
        return st;
    }
    OutArgs oa{};
    oa.wo = m.wo;
    oa.bo = m.bo;
    oa.has_bo = m.has_bo ? 1 : 0;
    oa.pre = m.y12;
    oa.beta = in.beta;
    oa.out = in.out;
    oa.part = m.opart;
    const float* A = m.xbuf;
    int lda = F * k;
    static const char* lnames[] = {"tower_layer1", "tower_layer2", "tower_layer3", "tower_layer4+"};
    for (size_t i = 0; i < m.layers.size(); ++i) {
      const bool last = i + 1 == m.layers.size();
      const DenseLayer& L = m.layers[i];
      float* C = m.h[i & 1];
      StageTimer t(m, s, lnames[std::min<size_t>(i, 3)]);
      if ((st = launch_tower_layer(s, L, B, A, lda, nullptr, C, L.Npad, last ? Epi::kOutput : Epi::kReluStore,
                                   last ? &oa : nullptr, nullptr, nullptr, true)))
        return st;
      A = C;
      lda = L.Npad;
    }
    return RMX_OK;
  }

  // DeepFM fp32 at a small launch batch: the whole tower + first order + FM + head in one launch, one block
  // per 16 samples (k_small_s3.hip; knob "s3_small")
  // (also the L-A path's staged rows, in.ids == nullptr: the kernel forms id = b F + f)
  if (m.type == RMX_MODEL_DEEPFM && !in.y1 && in.dtype == kF32 && !needs_gather_x(m) &&
      tower_small_s3_usable(m, B, F, k, true)) {
    StageTimer t(m, s, "tower_small");
    OutArgs oa{};
    oa.wo = m.wo;
    oa.bo = m.bo;
    oa.has_bo = m.has_bo ? 1 : 0;
    oa.beta = in.beta;
    oa.out = in.out;
    return launch_tower_small_s3(s, m, B, F, in.ids, (const float*)in.table, in.ld, (const float*)in.wtab, in.wld, oa);
  }

  // DeepFM fp32 at a batch that fills the GPU: the whole tower + first order + FM + head in one persistent
  // row-owner launch, h1 and h2 in registers (k_fused_s3.hip; knob "s3_fused")
  if (m.type == RMX_MODEL_DEEPFM && in.ids && !in.y1 && in.dtype == kF32 && !needs_gather_x(m) && k == 16 &&
      m.layers.size() == 3 && tower_fused_s3_usable(m.layers[0], m.layers[1], m.layers[2], B, F, k, true)) {
    StageTimer t(m, s, "tower_fused");
    OutArgs oa{};
    oa.wo = m.wo;
    oa.bo = m.bo;
    oa.has_bo = m.has_bo ? 1 : 0;
    oa.beta = in.beta;
    oa.out = in.out;
    return launch_tower_fused_s3(s, m.layers[0], m.layers[1], m.layers[2], B, F, in.ids, (const float*)in.table, in.ld,
                                 (const float*)in.wtab, in.wld, oa);
  }

  // 1. first order (+ FM for DeepFM; fused into tower layer 1 when it gathers through the split GEMM)
  const float* pre = nullptr;
  AGatherArgs ga{in.ids, (const float*)in.table, F, k, in.ld};
  bool gather_first = !needs_gather_x(m);
  // DeepFM on the split GEMM: first order + FM inside tower layer 1; the other models with a
  // gathered layer 1 (xDeepFM, DCN): the first order there
  const bool deepfm = m.type == RMX_MODEL_DEEPFM;
  const bool fm_fused = (deepfm || m.type == RMX_MODEL_XDEEPFM || m.type == RMX_MODEL_DCN) && !in.y1 &&
                        (!deepfm || in.dtype == kF32) && gather_first && m.layers.size() > 1 &&
                        tower_fm_fusable(m.layers[0], B, &ga, deepfm);
  // the first order by its own kernel (fm_y1 = 0, default) and the FM sums in layer 1: the sums are
  // free there, while summing the first-order weights in layer 1's epilogue exposes their gather
  // latency (bench: 0.213 ms layer 1 vs 0.022 + 0.172; DeepFM 154M -> 161M ex/s)
  // fm_y1: 0 = first-order kernel, 1 = layer 1's epilogue gathers, 2 (default) = summed from the
  // ring's weight DMAs when layer 1 runs a w-ring tile (free), else the first-order kernel
  const int fm_y1 = tuning_get("fm_y1", 2);
  // PNN bf16: its first order (a kernel of its own otherwise: nothing else gathers the weights) summed by
  // the tower tail's head (knob "tail_fo", default on)
  const size_t nl = m.layers.size();
  // DCN bf16 too when layer 1 does not sum it from its weight ring (tower_wring: the 2-deep ring variants)
  const bool tail_fo = (m.type == RMX_MODEL_PNN || (m.type == RMX_MODEL_DCN && !fm_fused)) && m.precision == kBF16 &&
                       in.dtype == kBF16 && in.ids && !in.y1 &&
                       F <= 40 && nl >= 3 && tuning_get("tail_fo", 1) != 0 &&
                       tower_tail_usable(m.layers[nl - 2], m.layers[nl - 1], B, m.layers[nl - 3].Npad);
  // DeepFM fp32 at a batch that fills the GPU: layer 1 + first order + FM as one row-owner kernel
  // (k_head_s3.hip; knob "s3_head")
  const bool head_s3 = deepfm && in.ids && !in.y1 && gather_first && in.dtype == kF32 && k == 16 &&
                       m.layers.size() > 1 && tower_head_s3_usable(m.layers[0], B, F, k, true);
  const bool fm_add = !head_s3 && fm_fused && deepfm &&
                      (fm_y1 == 0 || (fm_y1 == 2 && !tower_wring(m.layers[0], B, &ga)));
  if (fm_add) {
    StageTimer t(m, s, "first_order");
    if ((st = launch_encoder(s, 0, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr, nullptr, in.ld,
                             in.wld)))
      return st;
  }
  if (fm_fused || head_s3) {
    pre = m.y12;
  } else if (m.type == RMX_MODEL_DEEPFM) {
    StageTimer t(m, s, "encoder_fm");
    st = launch_encoder(s, in.y1 ? 3 : 1, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr, nullptr, in.ld,
                        in.wld);
    pre = m.y12;
  } else if (m.type != RMX_MODEL_DNN) {
    if (!in.y1 && !tail_fo) {
      StageTimer t(m, s, "first_order");
      st = launch_encoder(s, 0, B, in.ids, in.table, in.wtab, in.dtype, F, k, m.y12, nullptr, nullptr, in.ld, in.wld);
    }
    pre = tail_fo ? nullptr : m.y12;  // (the L-A irregular path already wrote y1 here)
  }
  if (st) return st;

  // 2. interaction encoders
  OutArgs oa{};
  oa.wo = m.wo;
  oa.bo = m.bo;
  oa.has_bo = m.has_bo ? 1 : 0;
  oa.pre = pre;
  oa.beta = in.beta;
  oa.out = in.out;
  oa.part = m.opart;
  const float* A = nullptr;
  int lda = 0;

  if (m.type == RMX_MODEL_XDEEPFM) {
    const float* uprev = nullptr;
    for (size_t l = 0; l < m.cin_layers.size(); ++l) {
      StageTimer t(m, s, l == 0 ? "cin_layer1" : (l == 1 ? "cin_layer2" : "cin_layer3+"));
      const bool last = l + 1 == m.cin_layers.size();
      float* uout = last ? nullptr : m.ubuf[l & 1];
      if ((st = launch_cin_layer(s, m.cin_layers[l], l == 0, last, B, F, k, in.ids, (const float*)in.table, uprev, uout,
                                 m.rowdot)))
        return st;
      uprev = uout;
    }
    oa.rowsum = m.rowdot;
    oa.rowsum_k = k;
  } else if (m.type == RMX_MODEL_DCN) {
    if (!m.dcn_fused) {
      StageTimer t(m, s, "cross");
      if ((st = launch_cross(s, B, F, k, m.cross_depth, in.ids, in.table, in.dtype, m.cross_w, m.cross_b, m.wo_x,
                             m.pre2)))
        return st;
    }
    oa.pre2 = m.pre2;
  } else if (m.type == RMX_MODEL_PNN) {
    StageTimer t(m, s, "product");
    if ((st = launch_product(s, B, F, k, in.ids, in.table, in.dtype, m.pairs, F * (F - 1) / 2, m.xbuf, m.precision,
                              xbuf_ld(m))))
      return st;
    A = m.xbuf;
    lda = xbuf_ld(m);
    gather_first = false;
  }
  if (m.type != RMX_MODEL_PNN && !gather_first) {
    StageTimer t(m, s, "gather_x");
    if ((st = launch_gather_x(s, B, F, k, in.ids, in.table, in.dtype, m.xbuf, m.precision, xbuf_ld(m))))
      return st;
    A = m.xbuf;
    lda = xbuf_ld(m);
  }

  // 3. tower (the last layer runs the output head: dot + bias + CAddTable + Sigmoid)
  static const char* names[] = {"tower_layer1", "tower_layer2", "tower_layer3", "tower_layer4+"};
  for (size_t i = 0; i < m.layers.size(); ++i) {
    const bool last = i + 1 == m.layers.size();
    const DenseLayer& L = m.layers[i];
    // bf16: the last hidden layer and the output layer in one persistent kernel (k_tail.hip)
    if (i >= 1 && i + 2 == m.layers.size() && m.precision == kBF16 &&
        tower_tail_usable(L, m.layers[i + 1], B, lda)) {
      StageTimer t(m, s, "tower_tail");
      const TailFirstOrder fo{in.ids, reinterpret_cast<const bf16_t*>(in.wtab), F, in.wld};
      return launch_tower_tail_bf16(s, L, m.layers[i + 1], B, reinterpret_cast<const bf16_t*>(A), lda, oa,
                                    tail_fo ? &fo : nullptr);
    }
    // fp32: the same pair on the split GEMM with h2 in registers (k_tail_s3.hip)
    if (i >= 1 && i + 2 == m.layers.size() && m.precision == kF32 && tower_tail_s3_usable(L, m.layers[i + 1], B, lda)) {
      StageTimer t(m, s, "tower_tail");
      return launch_tower_tail_s3(s, L, m.layers[i + 1], B, A, lda, oa);
    }
    float* C = m.h[i & 1];
    StageTimer t(m, s, names[std::min<size_t>(i, 3)]);
    if (i == 0 && head_s3) {
      if ((st = launch_tower_head_s3(s, L, B, F, in.ids, (const float*)in.table, in.ld, (const float*)in.wtab, in.wld, C,
                                     L.Npad, m.y12, 1)))
        return st;
      A = C;
      lda = L.Npad;
      continue;
    }
    XColArgs xc{m.xcol, L.N1, m.cross_depth + 1};
    FmArgs fm{in.wtab, in.dtype == kBF16 ? 1 : 0, deepfm ? 1 : 0, fm_add ? 1 : 0, m.y12, in.wld};
    st = launch_tower_layer(s, L, B, A, lda, (i == 0 && gather_first) ? &ga : nullptr, C, L.Npad,
                            last ? Epi::kOutput : Epi::kReluStore, last ? &oa : nullptr,
                            (i == 0 && m.dcn_fused) ? &xc : nullptr, (i == 0 && fm_fused) ? &fm : nullptr);
    if (st) return st;
    if (i == 0 && m.dcn_fused && (st = launch_cross_finish(s, B, m.cross_depth, m.xcol, m.cross_scalars, m.pre2)))
      return st;
    A = C;
    lda = L.Npad;
  }
  return RMX_OK;
}

// L-A: the reference's host-array contract.
// Stages the L-A host arrays on the device (mats packed, E / w uploaded, irregular first order
// precomputed) and describes them as one forward's inputs (implicit ids b*F + f).
int model_stage_host(rmx_model& m, int B, int64_t nnz, const int64_t* index, bool regular, bool sorted,
                     float bias, const float* weights, const float* embedding, const float* mats, FwdInputs* pin) {
  hipStream_t s = m.ctx->stream;
  int st;
  if (nnz > m.la_nnz) {
    RMX_HIP(hipDeviceSynchronize());
    dev_free(m.la_E);
    dev_free(m.la_w);
    if (m.type != RMX_MODEL_LR && (st = dev_alloc(&m.la_E, (size_t)nnz * m.k))) return st;
    if ((st = dev_alloc(&m.la_w, nnz))) return st;
    m.la_nnz = nnz;
  }
  if (B > m.la_B) {
    RMX_HIP(hipDeviceSynchronize());
    dev_free(m.la_out);
    dev_free(m.la_rowptr);
    if ((st = dev_alloc(&m.la_out, B))) return st;
    if (hipMalloc(&m.la_rowptr, sizeof(int64_t) * (B + 1)) != hipSuccess) {
      set_error("out of device memory");
      return RMX_E_NOMEM;
    }
    m.la_B = B;
  }
  if ((st = ensure_ws(m, B))) return st;
  {
    // the L-A contract hands over the whole mats array with every call (RecModel.scala:37-48; the reference
    // copies it into fresh BigDL modules per forward, LayerUtil.scala:13-19): H2D + pack, timed as la_mats
    StageTimer t(m, s, "la_mats");
    if (m.mats_len > 0 && (st = model_load_mats(m, mats, false))) return st;
  }
  // la_h2d: the gathered rows / weights (+ row pointers) to HBM; for bf16 models and irregular batches also
  // their rounding / the CSR first order that follows the copies
  StageTimer t_h2d(m, s, "la_h2d");
  // (the caller's pageable arrays go through the runtime's own staging copy: a pinned buffer filled by 1-16 host
  // threads beside the chunks' DMAs measured slower at B = 4,096 and 65,536, profiles/r06/ab_la_staging.txt)
  if (m.type != RMX_MODEL_LR && nnz > 0)
    RMX_HIP(hipMemcpyAsync(m.la_E, embedding, sizeof(float) * nnz * m.k, hipMemcpyHostToDevice, s));

  const bool use_w = m.type != RMX_MODEL_DNN;
  const bool csr = use_w && (m.type == RMX_MODEL_LR || !regular);
  if (use_w && nnz > 0) {
    if (csr && !sorted) {
      // stable counting sort by row keeps ascending-n order inside every row (Scatter order)
      m.h_rowptr.assign(B + 1, 0);
      for (int64_t n = 0; n < nnz; ++n) ++m.h_rowptr[(int32_t)index[n] + 1];
      for (int b = 0; b < B; ++b) m.h_rowptr[b + 1] += m.h_rowptr[b];
      std::vector<int64_t> pos(m.h_rowptr.begin(), m.h_rowptr.end() - 1);
      m.h_wperm.resize(nnz);
      for (int64_t n = 0; n < nnz; ++n) m.h_wperm[pos[(int32_t)index[n]]++] = weights[n];
      RMX_HIP(hipMemcpyAsync(m.la_w, m.h_wperm.data(), sizeof(float) * nnz, hipMemcpyHostToDevice, s));
    } else {
      RMX_HIP(hipMemcpyAsync(m.la_w, weights, sizeof(float) * nnz, hipMemcpyHostToDevice, s));
    }
  }
  if (m.precision == kBF16 && nnz > 0) {
    // a bf16 model reads the caller's fp32 arrays as a bf16 table: round them once on the device
    // (la_w in place too, so the Scatter first order below sums the rounded weights)
    if (nnz * std::max(m.k, 1) > m.la16_cap) {
      RMX_HIP(hipDeviceSynchronize());
      dev_free(m.la_E16);
      dev_free(m.la_w16);
      if (hipMalloc(&m.la_E16, sizeof(bf16_t) * nnz * std::max(m.k, 1)) != hipSuccess ||
          hipMalloc(&m.la_w16, sizeof(bf16_t) * nnz) != hipSuccess) {
        set_error("out of device memory");
        return RMX_E_NOMEM;
      }
      m.la16_cap = nnz * std::max(m.k, 1);
    }
    if (m.type != RMX_MODEL_LR && (st = launch_convert_bf16(s, m.la_E, nnz * m.k, m.la_E16))) return st;
    if (use_w) {
      if ((st = launch_convert_bf16(s, m.la_w, nnz, m.la_w16))) return st;
      if ((st = launch_widen_bf16(s, m.la_w16, nnz, m.la_w))) return st;
    }
  }
  if (csr) {
    if (sorted) {
      m.h_rowptr.assign(B + 1, 0);
      for (int64_t n = 0; n < nnz; ++n) ++m.h_rowptr[(int32_t)index[n] + 1];
      for (int b = 0; b < B; ++b) m.h_rowptr[b + 1] += m.h_rowptr[b];
    }
    RMX_HIP(hipMemcpyAsync(m.la_rowptr, m.h_rowptr.data(), sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, s));
    if ((st = launch_first_order_csr(s, B, m.la_rowptr, m.la_w, m.y12))) return st;
  }
  FwdInputs in;
  in.B = B;
  in.ids = nullptr;
  in.table = m.la_E;
  in.wtab = m.la_w;
  if (m.precision == kBF16) {
    in.table = m.la_E16;
    in.wtab = m.la_w16;
    in.dtype = kBF16;
  }
  in.y1 = csr ? m.y12 : nullptr;
  in.beta = bias;
  in.out = m.la_out;
  *pin = in;
  return RMX_OK;
}

int model_forward_host(rmx_model& m, int B, int64_t nnz, const int64_t* index, bool regular, bool sorted,
                       float bias, const float* weights, const float* embedding, const float* mats,
                       float* out) {
  hipStream_t s = m.ctx->stream;
  FwdInputs in;
  int st = model_stage_host(m, B, nnz, index, regular, sorted, bias, weights, embedding, mats, &in);
  if (st) return st;
  if ((st = model_forward(m, s, in))) return st;
  {
    StageTimer t(m, s, "la_d2h");
    RMX_HIP(hipMemcpyAsync(out, m.la_out, sizeof(float) * B, hipMemcpyDeviceToHost, s));
  }
  RMX_HIP(hipStreamSynchronize(s));
  // host buffers (h_rowptr / h_wperm) stay alive until the sync above
  return RMX_OK;
}

}  // namespace rmx
