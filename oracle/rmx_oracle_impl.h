/*
 * rmx_oracle_impl.h -- per-precision body of the oracle forward (TEST INFRASTRUCTURE ONLY).
 * Included twice by rmx_oracle.c with REAL = float and REAL = double.
 *
 * Activations of a block of RB samples are kept transposed ([feature][RB]) so
 * that each dot product is still summed sequentially over its input index (the
 * BigDL/MKL order is unknown; sequential is the documented choice) while the RB
 * independent rows vectorise.  No fast-math, no FMA contraction (see Makefile).
 */
#ifndef REAL
#error "define REAL and FN before including rmx_oracle_impl.h"
#endif

/* BigDL Linear (y = b + x W^T, W stored out x in row-major, util/LayerUtil.scala:7-26);
 * XT is [in][RB], YT is [out][RB].  relu: BigDL ReLU = Threshold(0, 0). */
static void FN(linear_rb)(int in, int out, const REAL* XT, const float* W, const float* b,
                          REAL* YT, int relu) {
  for (int n = 0; n < out; ++n) {
    const float* wn = W + (int64_t)n * in;
    REAL acc[RB];
    for (int r = 0; r < RB; ++r) acc[r] = 0;
    for (int i = 0; i < in; ++i) {
      const REAL wv = (REAL)wn[i];
      const REAL* xr = XT + (int64_t)i * RB;
      for (int r = 0; r < RB; ++r) acc[r] += xr[r] * wv;
    }
    for (int r = 0; r < RB; ++r) {
      REAL v = b ? acc[r] + (REAL)b[n] : acc[r];
      if (relu) v = v > 0 ? v : (REAL)0;
      YT[(int64_t)n * RB + r] = v;
    }
  }
}

/* precision 2 (bf16 emulation, f64 instantiation only): activations the device stores between
 * GEMM layers are rounded to bf16 (round to nearest even of the fp32 value); the last hidden layer
 * (consumed by the fused output dot in registers) stays unrounded.  See DESIGN.md §4, bf16 row. */
static REAL FN(act)(REAL v, int store) {
  if (!store || !g_bf16) return v;
  return (REAL)bf16_round((float)v);
}

static REAL FN(sigmoid)(REAL x) {
  /* BigDL Sigmoid: 1 / (1 + exp(-x)), exp through java.lang.Math.exp (double). */
  const REAL e = (REAL)exp(-(double)x);
  return (REAL)1 / ((REAL)1 + e);
}

/* x block: XT[d][r] = e[b0+r, d] (d = f*k + j, Reshape(B, F*k),
 * model/encoder/HigherOrderEncoder.scala:37); rows past B are zero. */
static void FN(load_x)(int B, int b0, int D, const float* E, REAL* XT) {
  for (int d = 0; d < D; ++d)
    for (int r = 0; r < RB; ++r)
      XT[(int64_t)d * RB + r] = (b0 + r < B) ? (REAL)E[(int64_t)(b0 + r) * D + d] : (REAL)0;
}

/* Tower T(x; dims) with optional output layer (model/encoder/HigherOrderEncoder.scala:34-59).
 * Consumes mats from *off; returns the final activation buffer (hidden width in *width). */
static REAL* FN(tower)(int in, const int32_t* fc, int n_fc, int with_output, const float* mats,
                       int64_t* off, REAL* XT, REAL* buf_a, REAL* buf_b, int* width) {
  REAL* cur = XT;
  int dim = in;
  for (int l = 0; l < n_fc; ++l) {
    REAL* nxt = (cur == buf_a) ? buf_b : buf_a;
    const float* W = mats + *off;
    const float* bb = W + (int64_t)dim * fc[l];
    FN(linear_rb)(dim, fc[l], cur, W, bb, nxt, 1);
    if (l + 1 < n_fc) /* stored between layers (bf16 mode) */
      for (int64_t i = 0; i < (int64_t)fc[l] * RB; ++i) nxt[i] = FN(act)(nxt[i], 1);
    *off += (int64_t)dim * fc[l] + fc[l];
    dim = fc[l];
    cur = nxt;
  }
  if (with_output) {
    REAL* nxt = (cur == buf_a) ? buf_b : buf_a;
    const float* W = mats + *off;
    FN(linear_rb)(dim, 1, cur, W, W + dim, nxt, 0);
    *off += (int64_t)dim + 1;
    dim = 1;
    cur = nxt;
  }
  *width = dim;
  return cur;
}

/* FM second order for one sample (model/encoder/SecondOrderEncoder.scala:19-34):
 * Sum(dim 2)->Power(2) minus Power(2)->Sum(dim 2), Mean over k, x0.5. */
static REAL FN(fm_one)(int F, int k, const float* e) {
  REAL acc = 0;
  for (int j = 0; j < k; ++j) {
    REAL s = 0, q = 0;
    for (int f = 0; f < F; ++f) {
      const REAL v = (REAL)e[(int64_t)f * k + j];
      s += v;
      q += v * v;
    }
    acc += s * s - q;
  }
  return (REAL)0.5 * (acc / (REAL)k);
}

static int FN(forward)(const orc_model* m, int B, const float* y1f, const float* bias,
                       const float* E, const float* mats, int nthreads, float* out) {
  const int F = m->n_fields, k = m->embedding_dim, D = F * k;
  const REAL beta = (REAL)bias[0];
  int maxw = D;
  for (int i = 0; i < m->n_fc; ++i) if (m->fc[i] > maxw) maxw = m->fc[i];
  for (int i = 0; i < m->n_cin; ++i) if (m->cin[i] > maxw) maxw = m->cin[i];
  if (m->type == ORC_PNN && F * (F - 1) / 2 > maxw) maxw = F * (F - 1) / 2;
  int cin_sum = 0, maxfc = 0;
  for (int i = 0; i < m->n_cin; ++i) cin_sum += m->cin[i];
  for (int i = 0; i < m->n_fc; ++i) if (m->fc[i] > maxfc) maxfc = m->fc[i];
  if (cin_sum + maxfc + D > maxw) maxw = cin_sum + maxfc + D;
  const int nblk = (B + RB - 1) / RB;

#pragma omp parallel num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
  {
    REAL* XT = (REAL*)malloc(sizeof(REAL) * ((size_t)maxw * RB * 4 + (size_t)2 * k * maxw) + 64);
    REAL* A = XT + (size_t)maxw * RB;
    REAL* Bf = A + (size_t)maxw * RB;
    REAL* C = Bf + (size_t)maxw * RB;
    REAL* UA = C + (size_t)maxw * RB;   /* CIN maps [j][h], two buffers */
    REAL* UB = UA + (size_t)k * maxw;
#pragma omp for schedule(dynamic, 1)
    for (int blk = 0; blk < nblk; ++blk) {
      const int b0 = blk * RB;
      REAL logit[RB];
      int64_t off = 0;
      int w = 0;
      if (m->type == ORC_LR) {
        /* model/lr/LR.scala:43-59: CAddTable(y1, bias) -> Sigmoid */
        for (int r = 0; r < RB; ++r) logit[r] = (b0 + r < B) ? (REAL)y1f[b0 + r] + beta : 0;
      } else if (m->type == ORC_DEEPFM || m->type == ORC_DNN) {
        /* model/deepfm/DeepFM.scala:54-80; model/dnn/DNN.scala:54-73 */
        FN(load_x)(B, b0, D, E, XT);
        REAL* y3 = FN(tower)(D, m->fc, m->n_fc, 1, mats, &off, XT, A, Bf, &w);
        for (int r = 0; r < RB; ++r) {
          if (b0 + r >= B) { logit[r] = 0; continue; }
          if (m->type == ORC_DEEPFM) {
            const REAL y2 = FN(fm_one)(F, k, E + (int64_t)(b0 + r) * D);
            REAL t = (REAL)y1f[b0 + r] + y2;   /* CAddTable: ((y1 + y2) + y3) + bias */
            t = t + y3[r];
            logit[r] = t + beta;
          } else {
            logit[r] = y3[r] + beta;
          }
        }
      } else if (m->type == ORC_XDEEPFM) {
        /* model/xdeepfm/CINEncoder.scala:36-58 (+ Appendix A semantics for L > 1). */
        FN(load_x)(B, b0, D, E, XT);
        REAL* d = FN(tower)(D, m->fc, m->n_fc, 0, mats, &off, XT, A, Bf, &w);
        const int dw = w;
        /* concat buffer C[c][r]: pooled CIN maps first, DNN hidden last (JoinTable(2,2), :167-171) */
        for (int c = 0; c < cin_sum + dw; ++c)
          for (int r = 0; r < RB; ++r) C[(int64_t)c * RB + r] = 0;
        for (int i = 0; i < dw; ++i)
          for (int r = 0; r < RB; ++r) C[(int64_t)(cin_sum + i) * RB + r] = d[(int64_t)i * RB + r];
        for (int r = 0; r < RB; ++r) {
          if (b0 + r >= B) continue;
          const float* e = E + (int64_t)(b0 + r) * D;
          int64_t coff = off;
          int pool_base = 0, Hp = F;
          /* per CIN layer over all j of this sample; u buffers are [j][h] in A / Bf */
          REAL* uprev = UA;
          for (int j = 0; j < k; ++j)
            for (int f = 0; f < F; ++f) uprev[(int64_t)j * maxw + f] = (REAL)e[(int64_t)f * k + j];
          for (int l = 0; l < m->n_cin; ++l) {
            const int H = m->cin[l];
            const float* Cw = mats + coff;          /* C_l: H x (F*Hp), :141 */
            const float* cb = Cw + (int64_t)H * F * Hp;
            REAL* ucur = (uprev == UA) ? UB : UA;
            for (int j = 0; j < k; ++j) {
              const REAL* up = uprev + (int64_t)j * maxw;
              for (int h2 = 0; h2 < H; ++h2) {
                const float* crow = Cw + (int64_t)h2 * F * Hp;
                REAL acc = 0;
                for (int f = 0; f < F; ++f) {
                  const REAL x0 = (REAL)e[(int64_t)f * k + j];
                  for (int h = 0; h < Hp; ++h) {
                    const REAL z = x0 * up[h];   /* MM(transB=true), :152 */
                    acc += z * (REAL)crow[(int64_t)f * Hp + h];
                  }
                }
                REAL v = acc + (REAL)cb[h2];
                ucur[(int64_t)j * maxw + h2] = v > 0 ? v : (REAL)0;   /* ReLU, :155 */
              }
            }
            /* pooling: Sum over k (:159-165) */
            for (int h2 = 0; h2 < H; ++h2) {
              REAL s = 0;
              for (int j = 0; j < k; ++j) s += ucur[(int64_t)j * maxw + h2];
              C[(int64_t)(pool_base + h2) * RB + r] = s;
            }
            pool_base += H;
            coff += (int64_t)H * F * Hp + H;
            Hp = H;
            uprev = ucur;
          }
        }
        for (int l = 0; l < m->n_cin; ++l) {
          const int Hp = l == 0 ? F : m->cin[l - 1];
          off += (int64_t)m->cin[l] * F * Hp + m->cin[l];
        }
        /* output Linear(sum(cinDims) + fc_last -> 1, no bias), :173-176 */
        REAL y[RB];
        {
          const float* Wo = mats + off;
          for (int r = 0; r < RB; ++r) y[r] = 0;
          for (int c = 0; c < cin_sum + dw; ++c)
            for (int r = 0; r < RB; ++r) y[r] += C[(int64_t)c * RB + r] * (REAL)Wo[c];
        }
        for (int r = 0; r < RB; ++r)
          logit[r] = (b0 + r < B) ? ((REAL)y1f[b0 + r] + y[r]) + beta : 0;  /* XDeepFM.scala:80-85 */
      } else if (m->type == ORC_DCN) {
        /* model/dcn/CrossEncoder.scala:40-55 */
        const int L = m->cross_depth;
        FN(load_x)(B, b0, D, E, XT);
        REAL* xl = C;  /* [d][r] */
        for (int64_t i = 0; i < (int64_t)D * RB; ++i) xl[i] = XT[i];
        const float* Wc = mats;               /* w_l: D each, :134-142 */
        const float* betas = mats + (int64_t)L * D;  /* beta_l: 1 each, :144-152 */
        for (int l = 0; l < L; ++l) {
          REAL s[RB];
          for (int r = 0; r < RB; ++r) s[r] = 0;
          for (int dd = 0; dd < D; ++dd)
            for (int r = 0; r < RB; ++r) s[r] += xl[(int64_t)dd * RB + r] * (REAL)Wc[(int64_t)l * D + dd];
          const REAL bl = (REAL)betas[l];
          for (int dd = 0; dd < D; ++dd)
            for (int r = 0; r < RB; ++r) {
              const int64_t ix = (int64_t)dd * RB + r;
              xl[ix] = ((XT[ix] * s[r]) + xl[ix]) + bl;   /* MM, CAddTable, CAdd: :46-48 */
            }
        }
        off = (int64_t)L * D + L;
        REAL* d = FN(tower)(D, m->fc, m->n_fc, 0, mats, &off, XT, A, Bf, &w);
        const float* Wo = mats + off;  /* Linear(D + fc_last -> 1, no bias), :176-185 */
        REAL y[RB];
        for (int r = 0; r < RB; ++r) y[r] = 0;
        for (int dd = 0; dd < D; ++dd)
          for (int r = 0; r < RB; ++r) y[r] += xl[(int64_t)dd * RB + r] * (REAL)Wo[dd];
        for (int i = 0; i < w; ++i)
          for (int r = 0; r < RB; ++r) y[r] += d[(int64_t)i * RB + r] * (REAL)Wo[D + i];
        for (int r = 0; r < RB; ++r)
          logit[r] = (b0 + r < B) ? ((REAL)y1f[b0 + r] + y[r]) + beta : 0;   /* DCN.scala:84-89 */
      } else { /* ORC_PNN: model/pnn/ProductEncoder.scala:34-41, model/pnn/PNN.scala:59-87 */
        const int P = F * (F - 1) / 2, D1 = m->fc[0];
        FN(load_x)(B, b0, D, E, XT);
        /* inner products, pairs (i<j) lexicographic (:110-120); Gather + DotProduct2 */
        REAL* IP = C;  /* [p][r] */
        for (int r = 0; r < RB; ++r) {
          int p = 0;
          for (int i = 0; i < F; ++i)
            for (int j2 = i + 1; j2 < F; ++j2, ++p) {
              REAL s = 0;
              if (b0 + r < B) {
                const float* e = E + (int64_t)(b0 + r) * D;
                for (int t = 0; t < k; ++t) s += (REAL)e[(int64_t)i * k + t] * (REAL)e[(int64_t)j2 * k + t];
              }
              IP[(int64_t)p * RB + r] = FN(act)(s, 1);  /* [x | ip] row stored for the GEMM */
            }
        }
        const float* Wz = mats;                        /* D1 x D, :78-82 */
        const float* Wp = mats + (int64_t)D * D1;      /* D1 x P, :91-95 */
        const float* bp = Wp + (int64_t)P * D1;        /* scalar, :104-108 */
        FN(linear_rb)(D, D1, XT, Wz, NULL, A, 0);
        FN(linear_rb)(P, D1, IP, Wp, NULL, Bf, 0);
        for (int64_t i = 0; i < (int64_t)D1 * RB; ++i) {
          const REAL v = (A[i] + Bf[i]) + (REAL)bp[0];   /* CAddTable, CAdd, ReLU: :97-102 */
          XT[i] = FN(act)(v > 0 ? v : (REAL)0, m->n_fc > 1);
        }
        off = (int64_t)D * D1 + (int64_t)P * D1 + 1;
        REAL* y = FN(tower)(D1, m->fc + 1, m->n_fc - 1, 1, mats, &off, XT, A, Bf, &w);
        for (int r = 0; r < RB; ++r)
          logit[r] = (b0 + r < B) ? ((REAL)y1f[b0 + r] + y[r]) + beta : 0;
      }
      for (int r = 0; r < RB; ++r)
        if (b0 + r < B) out[b0 + r] = (float)FN(sigmoid)(logit[r]);
    }
    free(XT);
  }
  return ORC_OK;
}
