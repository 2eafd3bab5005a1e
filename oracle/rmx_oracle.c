/*
 * rmx_oracle.c -- CPU restatement of the reference CTR forward path.
 * TEST INFRASTRUCTURE ONLY (see rmx_oracle.h header): parity unpinned, checked
 * against tests/ref_numpy.py and known-answer identities.
 */
#include "rmx_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#define RB 8

/* bf16 round-to-nearest-even of a finite fp32 value (v_cvt_pk_bf16_f32 for non-NaN inputs) */
static float bf16_round(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  u &= 0xFFFF0000u;
  memcpy(&f, &u, 4);
  return f;
}

/* precision-2 flag (set per orc_forward call; the oracle is test infrastructure, not thread-safe
 * across concurrent precision-2 and other calls) */
static int g_bf16 = 0;

/* ---------------------------------------------------------------- sizes ---- */

static void push_pair(int32_t* out, int32_t cap, int32_t* n, int32_t a, int32_t b) {
  if (*n + 2 <= cap) {
    out[*n] = a;
    out[*n + 1] = b;
  }
  *n += 2;
}

/* getMatsSize:
 *   LR       yr/model/lr/LR.scala:15                  (empty)
 *   DeepFM   yr/model/deepfm/DeepFM.scala:15-20       dims = [F*k] ++ fc ++ [1]; (in,out),(out,1)
 *   DNN      yr/model/dnn/DNN.scala:15-20             same as DeepFM
 *   xDeepFM  yr/model/xdeepfm/XDeepFM.scala:15-28     fc pairs ++ cin pairs ++ (sum(cin)+fc_last, 1)
 *   DCN      yr/model/dcn/DCN.scala:15-32             (D,1)*L ++ (1,1)*L ++ fc pairs ++ (D+fc_last, 1)
 *   PNN      yr/model/pnn/PNN.scala:15-25             (D,D1),(P,D1),(1,1) ++ pairs over fc ++ [1]  */
int32_t orc_mats_sizes(const orc_model* m, int32_t* out, int32_t cap) {
  int32_t n = 0;
  const int32_t F = m->n_fields, k = m->embedding_dim, D = F * k;
  switch (m->type) {
    case ORC_LR:
      break;
    case ORC_DEEPFM:
    case ORC_DNN: {
      int32_t prev = D;
      for (int i = 0; i <= m->n_fc; ++i) {
        const int32_t cur = i < m->n_fc ? m->fc[i] : 1;
        push_pair(out, cap, &n, prev, cur);
        push_pair(out, cap, &n, cur, 1);
        prev = cur;
      }
      break;
    }
    case ORC_XDEEPFM: {
      int32_t prev = D;
      for (int i = 0; i < m->n_fc; ++i) {
        push_pair(out, cap, &n, prev, m->fc[i]);
        push_pair(out, cap, &n, m->fc[i], 1);
        prev = m->fc[i];
      }
      int32_t hp = F, sum = 0;
      for (int i = 0; i < m->n_cin; ++i) {
        push_pair(out, cap, &n, F * hp, m->cin[i]);
        push_pair(out, cap, &n, m->cin[i], 1);
        hp = m->cin[i];
        sum += m->cin[i];
      }
      push_pair(out, cap, &n, sum + m->fc[m->n_fc - 1], 1);
      break;
    }
    case ORC_DCN: {
      for (int i = 0; i < m->cross_depth; ++i) push_pair(out, cap, &n, D, 1);
      for (int i = 0; i < m->cross_depth; ++i) push_pair(out, cap, &n, 1, 1);
      int32_t prev = D;
      for (int i = 0; i < m->n_fc; ++i) {
        push_pair(out, cap, &n, prev, m->fc[i]);
        push_pair(out, cap, &n, m->fc[i], 1);
        prev = m->fc[i];
      }
      push_pair(out, cap, &n, D + m->fc[m->n_fc - 1], 1);
      break;
    }
    case ORC_PNN: {
      const int32_t P = F * (F - 1) / 2;
      push_pair(out, cap, &n, D, m->fc[0]);
      push_pair(out, cap, &n, P, m->fc[0]);
      push_pair(out, cap, &n, 1, 1);
      int32_t prev = m->fc[0];
      for (int i = 1; i <= m->n_fc; ++i) {
        const int32_t cur = i < m->n_fc ? m->fc[i] : 1;
        push_pair(out, cap, &n, prev, cur);
        push_pair(out, cap, &n, cur, 1);
        prev = cur;
      }
      break;
    }
    default:
      return -1;
  }
  return n;
}

int64_t orc_mats_len(const orc_model* m) {
  int32_t sz[256];
  const int32_t n = orc_mats_sizes(m, sz, 256);
  if (n < 0 || n > 256) return -1;
  int64_t tot = 0;
  for (int i = 0; i < n; i += 2) tot += (int64_t)sz[i] * sz[i + 1];
  return tot;
}

/* ------------------------------------------------------------ synthetic ---- */

uint64_t orc_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

/* U(-a, a) from the top 24 bits; one exact int->float conversion and one rounding
 * multiply, so host and device produce the same bits. */
static float unif(uint64_t h, float a) {
  const float scale = a * (1.0f / 8388608.0f);
  return (float)((int32_t)(h >> 40) - 8388608) * scale;
}

void orc_gen_ids(uint64_t seed, int64_t row0, int32_t B, int32_t F, int64_t V, int32_t* ids) {
  const uint64_t per = (uint64_t)(V / F);
  for (int32_t b = 0; b < B; ++b)
    for (int32_t f = 0; f < F; ++f) {
      const uint64_t c = (uint64_t)(row0 + b) * (uint64_t)F + (uint64_t)f;
      ids[(int64_t)b * F + f] = (int32_t)((uint64_t)f * per + orc_splitmix64(seed ^ c) % per);
    }
}

void orc_gen_table(uint64_t seed, int64_t V, int32_t k, int64_t id0, int64_t nrows, float* w,
                   float* emb) {
  (void)V;
  for (int64_t r = 0; r < nrows; ++r) {
    const uint64_t id = (uint64_t)(id0 + r);
    const uint64_t base = id * (uint64_t)(k + 1);
    if (emb)
      for (int32_t j = 0; j < k; ++j) emb[r * k + j] = unif(orc_splitmix64(seed ^ (base + j)), 0.05f);
    if (w) w[r] = unif(orc_splitmix64(seed ^ (base + k)), 0.05f);
  }
}

/* Segment kinds: weight (Xavier over fan_in + fan_out) or bias (U(-0.01, 0.01)). */
static void fill_w(float* p, int64_t n, int32_t fin, int32_t fout, uint64_t seed, int64_t off) {
  const float a = sqrtf(6.0f / (float)(fin + fout));
  for (int64_t i = 0; i < n; ++i) p[i] = unif(orc_splitmix64(seed ^ (uint64_t)(off + i)), a);
}
static void fill_b(float* p, int64_t n, uint64_t seed, int64_t off) {
  for (int64_t i = 0; i < n; ++i) p[i] = unif(orc_splitmix64(seed ^ (uint64_t)(off + i)), 0.01f);
}

void orc_init_mats(const orc_model* m, uint64_t seed, float* mats) {
  int32_t sz[256];
  const int32_t n = orc_mats_sizes(m, sz, 256);
  const int32_t F = m->n_fields, k = m->embedding_dim, D = F * k;
  int64_t off = 0;
  int pair = 0;
  /* Which pairs are biases (vs weights) follows the LayerUtil calls of each model. */
  for (int i = 0; i < n; i += 2, ++pair) {
    const int32_t a = sz[i], b = sz[i + 1];
    const int64_t len = (int64_t)a * b;
    int is_bias = 0;
    switch (m->type) {
      case ORC_DEEPFM:
      case ORC_DNN:
        is_bias = pair & 1;
        break;
      case ORC_XDEEPFM: {
        const int nfc = 2 * m->n_fc, ncin = 2 * m->n_cin;
        if (pair < nfc) is_bias = pair & 1;
        else if (pair < nfc + ncin) is_bias = (pair - nfc) & 1;
        else is_bias = 0;
        break;
      }
      case ORC_DCN: {
        const int L = m->cross_depth, nfc = 2 * m->n_fc;
        if (pair < L) is_bias = 0;
        else if (pair < 2 * L) is_bias = 1;
        else if (pair < 2 * L + nfc) is_bias = (pair - 2 * L) & 1;
        else is_bias = 0;
        break;
      }
      case ORC_PNN:
        if (pair < 2) is_bias = 0;
        else if (pair == 2) is_bias = 1;
        else is_bias = (pair - 3) & 1;
        break;
      default:
        break;
    }
    if (is_bias) {
      fill_b(mats + off, len, seed, off);
    } else {
      /* Linear(in = a, out = b); a DCN cross vector is Linear(D -> 1). */
      fill_w(mats + off, len, a, b, seed, off);
    }
    off += len;
  }
  (void)D;
}

/* --------------------------------------------------------------- gather ---- */

int32_t orc_gather(int64_t V, int32_t k, const float* w_table, const float* emb_table, int32_t layout,
                   int64_t nnz, const int64_t* feats, float* w_out, float* emb_out) {
  for (int64_t n = 0; n < nnz; ++n) {
    /* ParRecModel.scala:282/:304: feats(i).toInt -- 32-bit truncation */
    const int32_t id = (int32_t)feats[n];
    if (id < 0 || id >= V) return ORC_E_INDEX;
    if (w_out) w_out[n] = w_table[id];
    if (emb_out)
      for (int32_t j = 0; j < k; ++j)
        emb_out[n * k + j] = layout == 0 ? emb_table[(int64_t)j * V + id] : emb_table[(int64_t)id * k + j];
  }
  return ORC_OK;
}

/* ---------------------------------------------------------- first order ---- */

/* bnn/Scatter.scala:17-36: output (B,1) zeroed, then output[index[i]] += w[i] for
 * ascending i, with require(index < batchSize). */
int32_t orc_first_order(int32_t B, int64_t nnz, const int64_t* index, const float* weights, float* y1) {
  for (int32_t b = 0; b < B; ++b) y1[b] = 0.0f;
  for (int64_t n = 0; n < nnz; ++n) {
    const int32_t ix = (int32_t)index[n];  /* DeepFM.scala:28 .map(_.toInt) */
    if (ix < 0 || ix >= B) return ORC_E_INDEX;
    y1[ix] += weights[n];
  }
  return ORC_OK;
}

/* ------------------------------------------------------ per-precision body -- */

#define REAL float
#define FN(x) x##_f32
#include "rmx_oracle_impl.h"
#undef REAL
#undef FN
#define REAL double
#define FN(x) x##_f64
#include "rmx_oracle_impl.h"
#undef REAL
#undef FN

void orc_round_bf16(int64_t n, const float* x, float* y) {
  for (int64_t i = 0; i < n; ++i) y[i] = bf16_round(x[i]);
}

int32_t orc_fm(int32_t B, int32_t F, int32_t k, const float* embedding, float* y2) {
  for (int32_t b = 0; b < B; ++b) y2[b] = fm_one_f32(F, k, embedding + (int64_t)b * F * k);
  return ORC_OK;
}

int32_t orc_forward(const orc_model* m, int32_t B, int64_t nnz, const int64_t* index, const float* bias,
                    const float* weights, const float* embedding, const float* mats, int32_t precision,
                    int32_t nthreads, float* out) {
  if (!m || B <= 0 || nnz < 0 || !bias || !out) return ORC_E_INVALID;
  if (m->type < ORC_LR || m->type > ORC_DNN) return ORC_E_INVALID;
  const int needs_emb = m->type != ORC_LR;
  const int needs_w = m->type != ORC_DNN;
  if (needs_emb) {
    if (!embedding || !mats) return ORC_E_INVALID;
    /* Reshape(Array(B, F, k), batchMode = false): nnz * k must equal B * F * k. */
    if (nnz != (int64_t)B * m->n_fields) return ORC_E_SHAPE;
  }
  float* y1 = (float*)calloc((size_t)B, sizeof(float));
  if (needs_w) {
    if (!weights || !index) { free(y1); return ORC_E_INVALID; }
    const int32_t st = orc_first_order(B, nnz, index, weights, y1);
    if (st != ORC_OK) { free(y1); return st; }
  }
  int32_t st;
  g_bf16 = precision == 2;
  if (precision >= 1)
    st = forward_f64(m, B, y1, bias, embedding, mats, nthreads, out);
  else
    st = forward_f32(m, B, y1, bias, embedding, mats, nthreads, out);
  free(y1);
  return st;
}
