/*
 * rmx_oracle.h -- CPU restatement of the reference's CTR forward path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (librmx.so, the rmx
 * Python package) links, loads or calls this code.  It is used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 *
 * PARITY STATUS: parity unpinned.  The reference (Scala 2.11 on BigDL 0.9.1 +
 * Angel 2.3.1, /root/reference/pom.xml:26-41) cannot be built or run here: no
 * JDK/Scala/Maven and no network.  The reference ships
 * no tests, fixtures or golden vectors.  This restatement is
 * pinned instead by (1) an independent numpy re-expression of the BigDL module
 * graphs in tests/ref_numpy.py, (2) known-answer identities (tests/), and
 * (3) the committed fixtures in tests/golden/ that both agree on.
 *
 * Every function cites the reference file:line it restates; paths are relative
 * to /root/reference/src/main/scala/, with io/yaochi/recommendation/ -> yr/ and
 * com/intel/analytics/bigdl/nn/ -> bnn/.
 */
#ifndef RMX_ORACLE_H
#define RMX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Model kinds: yr/model/{lr,deepfm,xdeepfm,dcn,pnn,dnn}/ */
enum {
  ORC_LR = 0,
  ORC_DEEPFM = 1,
  ORC_XDEEPFM = 2,
  ORC_DCN = 3,
  ORC_PNN = 4,
  ORC_DNN = 5
};

#define ORC_MAX_LAYERS 8

typedef struct {
  int32_t type;
  int32_t n_fields;              /* F  (nFields)       */
  int32_t embedding_dim;         /* k  (embeddingDim)  */
  int32_t n_fc;                  /* len(fcDims)        */
  int32_t fc[ORC_MAX_LAYERS];
  int32_t n_cin;                 /* len(cinDims)       */
  int32_t cin[ORC_MAX_LAYERS];
  int32_t cross_depth;           /* DCN crossDepth     */
} orc_model;

/* Status codes (mirror include/rmx.h). */
#define ORC_OK 0
#define ORC_E_INVALID (-1)
#define ORC_E_INDEX (-2)   /* bnn/Scatter.scala:29-30 require(index < batchSize) */
#define ORC_E_SHAPE (-3)   /* BigDL Reshape size mismatch (nnz != B*F)          */

/* getMatsSize (e.g. yr/model/deepfm/DeepFM.scala:15-20).  Returns the number of
 * int32 written (pairs * 2); writes nothing if cap is too small. */
int32_t orc_mats_sizes(const orc_model* m, int32_t* out, int32_t cap);
/* Flat mats length: sum over pairs of sizes[2i]*sizes[2i+1]
 * (yr/model/ParRecModel.scala:107-113). */
int64_t orc_mats_len(const orc_model* m);

/* ---- synthetic data; the device generator is bit-identical ---- */
uint64_t orc_splitmix64(uint64_t x);
/* Field-partitioned uniform ids: ids[b*F+f] = f*(V/F) + h(seed^((row0+b)*F+f)) % (V/F). */
void orc_gen_ids(uint64_t seed, int64_t row0, int32_t B, int32_t F, int64_t V, int32_t* ids);
/* Table init U(-0.05,0.05): emb row-major [V][k] (may be NULL) and w [V] (may be NULL). */
void orc_gen_table(uint64_t seed, int64_t V, int32_t k, int64_t id0, int64_t nrows,
                   float* w, float* emb_rowmajor);
/* mats init: Xavier-uniform weights, U(-0.01,0.01) biases, per model segment. */
void orc_init_mats(const orc_model* m, uint64_t seed, float* mats);

/* ---- gather (yr/model/ParRecModel.scala:279-284 makeWeights, :300-306 makeEmbeddings) ----
 * layout 0 = reference PS layout, coordinate-major k x V (Emb_j[id] = emb[j*V + id]);
 * layout 1 = row-major V x k.  Output E is nnz x k row-major, w_out is nnz. */
int32_t orc_gather(int64_t V, int32_t k, const float* w_table, const float* emb_table, int32_t layout,
                   int64_t nnz, const int64_t* feats, float* w_out, float* emb_out);

/* ---- forward (RecModel.forward, yr/model/RecModel.scala:37-48 -> buildParams :146-155) ----
 * Inputs are the reference's flat arrays: index[nnz] (COO row ids), the gathered
 * weights[nnz] and embedding[nnz*k], bias[1], mats.  precision 0 = fp32 in BigDL
 * op order, 1 = fp64 accumulation (for error bounds), 2 = fp64 accumulation with the bf16
 * storage points of a bf16 model emulated (activations stored between GEMM layers and the PNN
 * inner products rounded to bf16; the caller passes bf16-rounded table rows and mats).  nthreads <= 0 -> OpenMP default.
 * out[B] receives sigmoid probabilities. */
int32_t orc_forward(const orc_model* m, int32_t B, int64_t nnz, const int64_t* index,
                    const float* bias, const float* weights, const float* embedding,
                    const float* mats, int32_t precision, int32_t nthreads, float* out);

/* Stage outputs for debugging/parity of individual encoders (fp32 path):
 * y1[B] first order (Scatter), y2[B] FM second order (DeepFM only, else 0). */
int32_t orc_first_order(int32_t B, int64_t nnz, const int64_t* index, const float* weights, float* y1);
int32_t orc_fm(int32_t B, int32_t F, int32_t k, const float* embedding, float* y2);
/* ---- backward (RecModel.backward, yr/model/RecModel.scala:65-115; oracle/rmx_oracle_train.c) ----
 * Same inputs as orc_forward plus targets[B] (label > 0 -> 1).  Writes the gradients the
 * reference writes back into the caller's arrays (yr/util/GradUtil.scala, BackwardUtil.scala):
 * g_bias[1], g_weights[nnz], g_embedding[nnz*k], g_mats[mats_len], and the mean BCE loss.
 * f64 throughout; arrays a model type does not use may be NULL. */
int32_t orc_backward(const orc_model* m, int32_t B, int64_t nnz, const int64_t* index, const float* bias,
                     const float* weights, const float* embedding, const float* mats, const float* targets,
                     float* g_bias, float* g_weights, float* g_embedding, float* g_mats, double* loss_out);

/* bf16 round-to-nearest-even of n fp32 values (the device's v_cvt_pk_bf16_f32 for finite values) */
void orc_round_bf16(int64_t n, const float* x, float* y);

#ifdef __cplusplus
}
#endif
#endif
