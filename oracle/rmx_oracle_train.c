/*
 * rmx_oracle_train.c -- CPU restatement of RecModel.backward (TEST INFRASTRUCTURE ONLY).
 *
 * Nothing in the product links or calls this file; tests/ use it as the checker of the device
 * backward.  Per sample, in double precision, written for clarity (test sizes are small).
 *
 * PARITY STATUS: parity unpinned against the reference (BigDL 0.9.1 cannot run here; SURVEY.md
 * §8c).  Pinned instead by central finite differences of orc_forward's f64 path
 * (tests/test_train.py): every gradient below is the exact derivative of the forward the oracle
 * already restates.
 *
 * Reference call sites (paths relative to /root/reference/src/main/scala/, yr/ =
 * io/yaochi/recommendation/, bnn/ = com/intel/analytics/bigdl/nn/):
 *   loss + output grads   yr/model/deepfm/DeepFM.scala:83-124 (BCECriterion, CAddTable, Sigmoid;
 *                         same pattern in lr/LR.scala:60-92, dnn/DNN.scala, dcn/DCN.scala,
 *                         pnn/PNN.scala, xdeepfm/XDeepFM.scala)
 *   targets               label > 0 -> 1 else 0 (DeepFM.scala:106)
 *   first order           bnn/Scatter.scala:38-59 (grad of w[n] = grad of row index[n])
 *   FM                    yr/model/encoder/SecondOrderEncoder.scala (module chain backward)
 *   tower                 yr/model/encoder/HigherOrderEncoder.scala:22-31 (Linear/ReLU backward),
 *                         yr/util/BackwardUtil.scala:6-30 (gradWeight, gradBias into mats)
 *   CIN                   yr/model/xdeepfm/CINEncoder.scala:60-103
 *   cross                 yr/model/dcn/CrossEncoder.scala:57-105
 *   product               yr/model/pnn/ProductEncoder.scala:43-70
 *   write-back            yr/util/GradUtil.scala:7-42 (weights, bias, embedding = sum of the
 *                         encoders' embedding grads)
 * BigDL BCECriterion (third-party, published algorithm; sizeAverage = true, eps = 1e-12):
 *   loss = -(1/B) sum_b [t log(p + eps) + (1 - t) log(1 - p + eps)]
 *   dL/dp = -(t - p) / ((1 - p + eps)(p + eps)) / B;  Sigmoid backward: g * (1 - p) * p.
 * CAddTable's broadcast scalar bias input receives the sum of the output gradient.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rmx_oracle.h"

#define EPS_BCE 1e-12

static double relu_d(double v) { return v > 0 ? v : 0.0; }

/* Hidden tower layers on x (dims in -> fc[0] -> ... ), activations acts[l][.] (post ReLU). */
static void tower_fwd(int in, const int32_t* fc, int n_fc, const float* mats, int64_t off, const double* x,
                      double** acts) {
  const double* cur = x;
  int dim = in;
  for (int l = 0; l < n_fc; ++l) {
    const float* W = mats + off;
    const float* b = W + (int64_t)dim * fc[l];
    for (int n = 0; n < fc[l]; ++n) {
      double a = 0;
      for (int i = 0; i < dim; ++i) a += cur[i] * (double)W[(int64_t)n * dim + i];
      acts[l][n] = relu_d(a + (double)b[n]);
    }
    off += (int64_t)dim * fc[l] + fc[l];
    dim = fc[l];
    cur = acts[l];
  }
}

/* Backward of tower_fwd given g_top = dL/d(acts[n_fc-1]) (overwritten); adds the Linear grads
 * into gm and writes dL/dx into gx (length in). */
static void tower_bwd(int in, const int32_t* fc, int n_fc, const float* mats, int64_t off0, const double* x,
                      double** acts, double* g_top, double* gm, double* gx, double* scratch) {
  int64_t offs[ORC_MAX_LAYERS];
  int64_t off = off0;
  int dim = in;
  for (int l = 0; l < n_fc; ++l) {
    offs[l] = off;
    off += (int64_t)dim * fc[l] + fc[l];
    dim = fc[l];
  }
  double* g = g_top;
  for (int l = n_fc - 1; l >= 0; --l) {
    const int K = l == 0 ? in : fc[l - 1];
    const double* inp = l == 0 ? x : acts[l - 1];
    const float* W = mats + offs[l];
    double* gW = gm + offs[l];
    double* gb = gW + (int64_t)K * fc[l];
    double* gin = l == 0 ? gx : scratch;
    for (int i = 0; i < K; ++i) gin[i] = 0;
    for (int n = 0; n < fc[l]; ++n) {
      const double gp = acts[l][n] > 0 ? g[n] : 0.0;  /* ReLU backward */
      if (gp == 0.0) continue;
      gb[n] += gp;
      for (int i = 0; i < K; ++i) {
        gW[(int64_t)n * K + i] += gp * inp[i];
        gin[i] += gp * (double)W[(int64_t)n * K + i];
      }
    }
    if (l > 0) {
      for (int i = 0; i < K; ++i) g_top[i] = gin[i];  /* reuse g_top storage as the next g */
      g = g_top;
    }
  }
  if (n_fc == 0)
    for (int i = 0; i < in; ++i) gx[i] = g_top[i];
}

static double sigmoid_d(double x) { return 1.0 / (1.0 + exp(-x)); }

int32_t orc_backward(const orc_model* m, int32_t B, int64_t nnz, const int64_t* index, const float* bias,
                     const float* weights, const float* embedding, const float* mats, const float* targets,
                     float* g_bias, float* g_weights, float* g_embedding, float* g_mats, double* loss_out) {
  if (!m || B <= 0 || nnz < 0 || !bias || !targets || !g_bias || !loss_out) return ORC_E_INVALID;
  const int F = m->n_fields, k = m->embedding_dim, D = F * k;
  const int needs_emb = m->type != ORC_LR;
  const int needs_w = m->type != ORC_DNN;
  if (needs_emb && (!embedding || !mats || !g_embedding || !g_mats || nnz != (int64_t)B * F)) return ORC_E_SHAPE;
  if (needs_w && (!weights || !index || !g_weights)) return ORC_E_INVALID;
  for (int64_t n = 0; n < nnz && needs_w; ++n)
    if (index[n] < 0 || index[n] >= B) return ORC_E_INDEX;
  const int64_t ML = needs_emb ? orc_mats_len(m) : 0;
  double* gm = (double*)calloc((size_t)(ML > 0 ? ML : 1), sizeof(double));
  double* y1 = (double*)calloc((size_t)B, sizeof(double));
  double* gz = (double*)calloc((size_t)B, sizeof(double));
  for (int64_t n = 0; n < nnz && needs_w; ++n) y1[index[n]] += (double)weights[n];

  int maxw = D + 1;
  for (int i = 0; i < m->n_fc; ++i) if (m->fc[i] > maxw) maxw = m->fc[i];
  int cin_sum = 0;
  for (int i = 0; i < m->n_cin; ++i) { cin_sum += m->cin[i]; if (m->cin[i] > maxw) maxw = m->cin[i]; }
  const int P = F * (F - 1) / 2;
  if (P > maxw) maxw = P;
  double* acts_mem = (double*)calloc((size_t)ORC_MAX_LAYERS * maxw, sizeof(double));
  double* acts[ORC_MAX_LAYERS];
  for (int l = 0; l < ORC_MAX_LAYERS; ++l) acts[l] = acts_mem + (size_t)l * maxw;
  double* x = (double*)calloc((size_t)maxw, sizeof(double));
  double* gx = (double*)calloc((size_t)maxw, sizeof(double));
  double* gx2 = (double*)calloc((size_t)maxw, sizeof(double));
  double* gt = (double*)calloc((size_t)maxw, sizeof(double));
  double* scr = (double*)calloc((size_t)maxw, sizeof(double));
  /* DCN cross states x_0..x_L, PNN ip / h0, CIN maps */
  const int L = m->cross_depth > 0 ? m->cross_depth : 0;
  double* xs = (double*)calloc((size_t)(L + 1) * D + 1, sizeof(double));
  double* sl = (double*)calloc((size_t)L + 1, sizeof(double));
  double* ip = (double*)calloc((size_t)P + 1, sizeof(double));
  double* h0 = (double*)calloc((size_t)(m->n_fc > 0 ? m->fc[0] : 1), sizeof(double));
  const int nc = m->n_cin;
  double* u = (double*)calloc((size_t)(nc + 1) * k * (maxw + F) + 1, sizeof(double));
  double* gu = (double*)calloc((size_t)(nc + 1) * k * (maxw + F) + 1, sizeof(double));
  double* pool = (double*)calloc((size_t)cin_sum + 1, sizeof(double));
  const int US = maxw + F;  /* u row stride */
  double loss = 0, gbias = 0;
  double* ge = (double*)calloc((size_t)D + 1, sizeof(double));

  for (int pass = 0; pass < 2; ++pass) {
    /* pass 0: forward -> loss, dL/dz;  pass 1: backward per sample */
    for (int b = 0; b < B; ++b) {
      const float* e = needs_emb ? embedding + (int64_t)b * D : NULL;
      for (int d = 0; d < D && needs_emb; ++d) x[d] = (double)e[d];
      double z = 0;
      const double beta = (double)bias[0];
      if (m->type == ORC_LR) {
        z = y1[b] + beta;
        if (pass == 1) { gbias += gz[b]; }
      } else if (m->type == ORC_DEEPFM || m->type == ORC_DNN) {
        tower_fwd(D, m->fc, m->n_fc, mats, 0, x, acts);
        int64_t off = 0;
        int dim = D;
        for (int l = 0; l < m->n_fc; ++l) { off += (int64_t)dim * m->fc[l] + m->fc[l]; dim = m->fc[l]; }
        const double* hL = m->n_fc ? acts[m->n_fc - 1] : x;
        double y3 = (double)mats[off + dim];
        for (int i = 0; i < dim; ++i) y3 += hL[i] * (double)mats[off + i];
        double y2 = 0;
        if (m->type == ORC_DEEPFM) {
          double acc = 0;
          for (int j = 0; j < k; ++j) {
            double s = 0, q = 0;
            for (int f = 0; f < F; ++f) { s += x[f * k + j]; q += x[f * k + j] * x[f * k + j]; }
            acc += s * s - q;
          }
          y2 = 0.5 * (acc / k);
          z = y1[b] + y2 + y3 + beta;
        } else {
          z = y3 + beta;
        }
        if (pass == 1) {
          const double g = gz[b];
          gbias += g;
          for (int i = 0; i < dim; ++i) { gm[off + i] += g * hL[i]; gt[i] = g * (double)mats[off + i]; }
          gm[off + dim] += g;
          tower_bwd(D, m->fc, m->n_fc, mats, 0, x, acts, gt, gm, gx, scr);
          for (int d = 0; d < D; ++d) ge[d] = gx[d];
          if (m->type == ORC_DEEPFM)
            for (int j = 0; j < k; ++j) {
              double s = 0;
              for (int f = 0; f < F; ++f) s += x[f * k + j];
              for (int f = 0; f < F; ++f) ge[f * k + j] += g * (s - x[f * k + j]) / k;
            }
        }
      } else if (m->type == ORC_DCN) {
        for (int d = 0; d < D; ++d) xs[d] = x[d];
        for (int l = 0; l < L; ++l) {
          double s = 0;
          for (int d = 0; d < D; ++d) s += xs[(int64_t)l * D + d] * (double)mats[(int64_t)l * D + d];
          sl[l] = s;
          for (int d = 0; d < D; ++d)
            xs[(int64_t)(l + 1) * D + d] = x[d] * s + xs[(int64_t)l * D + d] + (double)mats[(int64_t)L * D + l];
        }
        const int64_t toff = (int64_t)L * D + L;
        tower_fwd(D, m->fc, m->n_fc, mats, toff, x, acts);
        int64_t off = toff;
        int dim = D;
        for (int l = 0; l < m->n_fc; ++l) { off += (int64_t)dim * m->fc[l] + m->fc[l]; dim = m->fc[l]; }
        const double* dh = acts[m->n_fc - 1];
        double y = 0;
        for (int d = 0; d < D; ++d) y += xs[(int64_t)L * D + d] * (double)mats[off + d];
        for (int i = 0; i < dim; ++i) y += dh[i] * (double)mats[off + D + i];
        z = y1[b] + y + beta;
        if (pass == 1) {
          const double g = gz[b];
          gbias += g;
          for (int d = 0; d < D; ++d) gm[off + d] += g * xs[(int64_t)L * D + d];
          for (int i = 0; i < dim; ++i) { gm[off + D + i] += g * dh[i]; gt[i] = g * (double)mats[off + D + i]; }
          tower_bwd(D, m->fc, m->n_fc, mats, toff, x, acts, gt, gm, gx, scr);
          /* cross stack backward: g_{l+1} -> g_l */
          double* gl = gx2;
          for (int d = 0; d < D; ++d) gl[d] = g * (double)mats[off + d];
          for (int d = 0; d < D; ++d) ge[d] = gx[d];
          for (int l = L - 1; l >= 0; --l) {
            double gs = 0, gb = 0;
            for (int d = 0; d < D; ++d) { gs += gl[d] * x[d]; gb += gl[d]; }
            gm[(int64_t)L * D + l] += gb;
            for (int d = 0; d < D; ++d) {
              ge[d] += gl[d] * sl[l];
              gm[(int64_t)l * D + d] += gs * xs[(int64_t)l * D + d];
            }
            for (int d = 0; d < D; ++d) gl[d] = gl[d] + gs * (double)mats[(int64_t)l * D + d];
          }
          for (int d = 0; d < D; ++d) ge[d] += gl[d];  /* x_0 = e */
        }
      } else if (m->type == ORC_PNN) {
        const int D1 = m->fc[0];
        int p = 0;
        for (int i = 0; i < F; ++i)
          for (int j2 = i + 1; j2 < F; ++j2, ++p) {
            double s = 0;
            for (int t = 0; t < k; ++t) s += x[i * k + t] * x[j2 * k + t];
            ip[p] = s;
          }
        const float* Wz = mats;
        const float* Wp = mats + (int64_t)D * D1;
        const double bp = (double)mats[(int64_t)D * D1 + (int64_t)P * D1];
        for (int n = 0; n < D1; ++n) {
          double a = 0, c = 0;
          for (int d = 0; d < D; ++d) a += x[d] * (double)Wz[(int64_t)n * D + d];
          for (int q = 0; q < P; ++q) c += ip[q] * (double)Wp[(int64_t)n * P + q];
          h0[n] = relu_d(a + c + bp);
        }
        const int64_t toff = (int64_t)D * D1 + (int64_t)P * D1 + 1;
        tower_fwd(D1, m->fc + 1, m->n_fc - 1, mats, toff, h0, acts);
        int64_t off = toff;
        int dim = D1;
        for (int l = 1; l < m->n_fc; ++l) { off += (int64_t)dim * m->fc[l] + m->fc[l]; dim = m->fc[l]; }
        const double* hL = m->n_fc > 1 ? acts[m->n_fc - 2] : h0;
        double y = (double)mats[off + dim];
        for (int i = 0; i < dim; ++i) y += hL[i] * (double)mats[off + i];
        z = y1[b] + y + beta;
        if (pass == 1) {
          const double g = gz[b];
          gbias += g;
          for (int i = 0; i < dim; ++i) { gm[off + i] += g * hL[i]; gt[i] = g * (double)mats[off + i]; }
          gm[off + dim] += g;
          double* gh0 = gx2;
          tower_bwd(D1, m->fc + 1, m->n_fc - 1, mats, toff, h0, acts, gt, gm, gh0, scr);
          double* gip = scr;  /* tower_bwd is done with scr */
          for (int q = 0; q < P; ++q) gip[q] = 0;
          for (int d = 0; d < D; ++d) ge[d] = 0;
          double gbp = 0;
          for (int n = 0; n < D1; ++n) {
            const double gp = h0[n] > 0 ? gh0[n] : 0.0;
            if (gp == 0.0) continue;
            gbp += gp;
            for (int d = 0; d < D; ++d) {
              gm[(int64_t)n * D + d] += gp * x[d];
              ge[d] += gp * (double)Wz[(int64_t)n * D + d];
            }
            for (int q = 0; q < P; ++q) {
              gm[(int64_t)D * D1 + (int64_t)n * P + q] += gp * ip[q];
              gip[q] += gp * (double)Wp[(int64_t)n * P + q];
            }
          }
          gm[(int64_t)D * D1 + (int64_t)P * D1] += gbp;
          p = 0;
          for (int i = 0; i < F; ++i)
            for (int j2 = i + 1; j2 < F; ++j2, ++p)
              for (int t = 0; t < k; ++t) {
                ge[i * k + t] += gip[p] * x[j2 * k + t];
                ge[j2 * k + t] += gip[p] * x[i * k + t];
              }
        }
      } else { /* ORC_XDEEPFM */
        tower_fwd(D, m->fc, m->n_fc, mats, 0, x, acts);
        int64_t off = 0;
        int dim = D;
        for (int l = 0; l < m->n_fc; ++l) { off += (int64_t)dim * m->fc[l] + m->fc[l]; dim = m->fc[l]; }
        const double* dh = acts[m->n_fc - 1];
        /* u_0[j][f] = x0[j][f] = e[f][j]; layer maps u_l[j][h] at u + l*k*US */
        for (int j = 0; j < k; ++j)
          for (int f = 0; f < F; ++f) u[(int64_t)j * US + f] = x[f * k + j];
        int64_t coff[ORC_MAX_LAYERS];
        int64_t co = off;
        int pb = 0;
        for (int l = 0; l < nc; ++l) {
          const int H = m->cin[l], Hp = l == 0 ? F : m->cin[l - 1];
          coff[l] = co;
          const float* Cw = mats + co;
          const float* cb = Cw + (int64_t)H * F * Hp;
          const double* up = u + (int64_t)l * k * US;
          double* uc = u + (int64_t)(l + 1) * k * US;
          for (int j = 0; j < k; ++j)
            for (int h2 = 0; h2 < H; ++h2) {
              double a = 0;
              for (int f = 0; f < F; ++f)
                for (int h = 0; h < Hp; ++h)
                  a += x[f * k + j] * up[(int64_t)j * US + h] * (double)Cw[(int64_t)h2 * F * Hp + (int64_t)f * Hp + h];
              uc[(int64_t)j * US + h2] = relu_d(a + (double)cb[h2]);
            }
          for (int h2 = 0; h2 < H; ++h2) {
            double s = 0;
            for (int j = 0; j < k; ++j) s += uc[(int64_t)j * US + h2];
            pool[pb + h2] = s;
          }
          pb += H;
          co += (int64_t)H * F * Hp + H;
        }
        const int64_t wo = co;
        double y = 0;
        for (int c = 0; c < cin_sum; ++c) y += pool[c] * (double)mats[wo + c];
        for (int i = 0; i < dim; ++i) y += dh[i] * (double)mats[wo + cin_sum + i];
        z = y1[b] + y + beta;
        if (pass == 1) {
          const double g = gz[b];
          gbias += g;
          for (int c = 0; c < cin_sum; ++c) gm[wo + c] += g * pool[c];
          for (int i = 0; i < dim; ++i) { gm[wo + cin_sum + i] += g * dh[i]; gt[i] = g * (double)mats[wo + cin_sum + i]; }
          tower_bwd(D, m->fc, m->n_fc, mats, 0, x, acts, gt, gm, gx, scr);
          for (int d = 0; d < D; ++d) ge[d] = gx[d];
          memset(gu, 0, sizeof(double) * (size_t)(nc + 1) * k * US);
          pb = cin_sum;
          for (int l = nc - 1; l >= 0; --l) {
            const int H = m->cin[l], Hp = l == 0 ? F : m->cin[l - 1];
            pb -= H;
            const float* Cw = mats + coff[l];
            double* gC = gm + coff[l];
            double* gc = gC + (int64_t)H * F * Hp;
            const double* up = u + (int64_t)l * k * US;
            const double* uc = u + (int64_t)(l + 1) * k * US;
            double* gup = gu + (int64_t)l * k * US;
            double* guc = gu + (int64_t)(l + 1) * k * US;
            for (int j = 0; j < k; ++j)
              for (int h2 = 0; h2 < H; ++h2) {
                const double gpre = uc[(int64_t)j * US + h2] > 0
                                        ? guc[(int64_t)j * US + h2] + g * (double)mats[wo + pb + h2]
                                        : 0.0;
                if (gpre == 0.0) continue;
                gc[h2] += gpre;
                for (int f = 0; f < F; ++f)
                  for (int h = 0; h < Hp; ++h) {
                    const double x0 = x[f * k + j], uv = up[(int64_t)j * US + h];
                    const double cw = (double)Cw[(int64_t)h2 * F * Hp + (int64_t)f * Hp + h];
                    gC[(int64_t)h2 * F * Hp + (int64_t)f * Hp + h] += gpre * x0 * uv;
                    ge[f * k + j] += gpre * cw * uv;        /* through x0 */
                    gup[(int64_t)j * US + h] += gpre * cw * x0;  /* through u_{l-1} */
                  }
              }
          }
          for (int j = 0; j < k; ++j)  /* u_0 = x0 */
            for (int f = 0; f < F; ++f) ge[f * k + j] += gu[(int64_t)j * US + f];
        }
      }
      if (pass == 0) {
        const double p = sigmoid_d(z);
        const double t = targets[b] > 0 ? 1.0 : 0.0;
        loss += -(t * log(p + EPS_BCE) + (1 - t) * log(1 - p + EPS_BCE));
        const double gp = -(t - p) / ((1 - p + EPS_BCE) * (p + EPS_BCE)) / B;
        gz[b] = gp * (1 - p) * p;
      } else if (needs_emb) {
        for (int d = 0; d < D; ++d) g_embedding[(int64_t)b * D + d] = (float)ge[d];
      }
    }
  }
  for (int64_t n = 0; n < nnz && needs_w; ++n) g_weights[n] = (float)gz[index[n]];
  g_bias[0] = (float)gbias;
  for (int64_t i = 0; i < ML; ++i) g_mats[i] = (float)gm[i];
  *loss_out = loss / B;
  free(gm); free(y1); free(gz); free(acts_mem); free(x); free(gx); free(gx2); free(gt); free(scr);
  free(xs); free(sl); free(ip); free(h0); free(u); free(gu); free(pool); free(ge);
  return ORC_OK;
}
