/*
 * rmx_jni.c -- thin JNI shim from the reference's Scala RecModel plugin API to librmx.so.
 *
 * The reference calls `RecModel.forward / backward(batchSize, batch, bias, weights, embeddings,
 * embeddingDim, mats, matSizes[, fields][, targets])` (src/main/scala/io/yaochi/recommendation/model/
 * RecModel.scala:9-115) from ParRecModel.predict / optimize (model/ParRecModel.scala:365-581), after
 * pulling and gathering the PS rows (pull* :165-199, make* :270-306).  A Scala object
 * `io.yaochi.recommendation.model.gpu.GpuRecModel` declares the natives below.
 *
 *   L-A (host arrays, the exact RecModel contract):   forward0, backward0
 *   L-B (HBM-resident table, replaces pull + make*):  createContext, createTable, uploadTable,
 *        fillTableSynthetic, setMats, setBias, setPrecision, forwardIds, backwardIds, predictIds, auc
 *   sharded table (RCCL, one rank per GPU):            commUniqueId, createShard, fillShardSynthetic,
 *        forwardIdsSharded, setShardOwnerHash
 *
 * A model handle is a `jmodel`: the rmx_model plus device staging for the L-B calls (ids, outputs,
 * targets, gradients), grown on demand and guarded by a mutex, so host int[] ids reach the device
 * with one copy per call.  librmx's own entry points are reentrant (include/rmx.h, rmx::ModelUse),
 * so Spark local[N] tasks may share one model.
 * Array access: GetPrimitiveArrayCritical for one synchronous call (no copy on HotSpot); nothing
 * calls back into the JVM while a critical section is open.  Errors become Java exceptions with the
 * reference's types:
 *   RMX_E_INDEX / RMX_E_INVALID -> IllegalArgumentException   (bnn/Scatter.scala:29-30 require)
 *   RMX_E_SHAPE / RMX_E_MATS    -> IllegalArgumentException   (BigDL Reshape size mismatch)
 *   RMX_E_TYPE                  -> scala.MatchError is not reachable from C: IllegalStateException
 *   RMX_E_HIP / RMX_E_NOMEM / RMX_E_COMM -> RuntimeException
 *
 * Build (needs a JDK; this container and the GPU box have none, so it is not built here --
 * tests/test_jni_shim.py compiles it against the JNI declarations it uses, syntax only):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *      rmx_jni.c -L../csrc -lrmx -lpthread -Wl,-rpath,'$ORIGIN' -o librmx_jni.so
 */
#if defined(__has_include)
#if __has_include(<jni.h>)
#define RMX_HAVE_JNI 1
#endif
#endif

#ifdef RMX_HAVE_JNI
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/rmx.h"

#define JFN(name) Java_io_yaochi_recommendation_model_gpu_GpuRecModel_##name

static void throw_status(JNIEnv* env, int st) {
  const char* cls = "java/lang/RuntimeException";
  if (st == RMX_E_INDEX || st == RMX_E_INVALID || st == RMX_E_SHAPE || st == RMX_E_MATS)
    cls = "java/lang/IllegalArgumentException";
  else if (st == RMX_E_TYPE)
    cls = "java/lang/IllegalStateException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, rmx_last_error());
}

/* The reference's require(...) on an argument (IllegalArgumentException, bnn/Scatter.scala:29-30):
 * every L-B native checks the Java arrays' lengths against what librmx will read or write BEFORE
 * staging anything, so a short or null array never reaches the device or a host copy. */
static int require_arg(JNIEnv* env, int ok, const char* msg) {
  if (ok) return 1;
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
  return 0;
}

static jlong alen(JNIEnv* env, jarray a) { return a ? (jlong)(*env)->GetArrayLength(env, a) : -1; }

/* ---- model handle: rmx_model + device staging for the L-B calls ---- */
typedef struct {
  rmx_model* m;
  rmx_ctx* ctx;          /* the model's context (NULL: metadata-only model) */
  int n_fields, k;       /* F and k of the model: the L-B array lengths are checked against them */
  pthread_mutex_t mu;    /* guards the staging buffers */
  void* d_ids;           /* int32 [cap_ids] */
  void* d_f;             /* float [cap_f]: outputs / targets / gradients, carved per call */
  size_t cap_ids, cap_f;
} jmodel;

static jmodel* JM(jlong h) { return (jmodel*)(intptr_t)h; }

static int grow(rmx_ctx* ctx, void** p, size_t* cap, size_t need, size_t es) {
  if (need <= *cap) return RMX_OK;
  if (*p) rmx_free(ctx, *p);
  *p = NULL;
  *cap = 0;
  int st = rmx_malloc(ctx, need * es, p);
  if (st == RMX_OK) *cap = need;
  return st;
}

/* long createContext(int device) / void destroyContext(long ctx) */
JNIEXPORT jlong JNICALL JFN(createContext)(JNIEnv* env, jclass cls, jint device) {
  (void)cls;
  rmx_ctx* c = NULL;
  int st = rmx_ctx_create(device, &c);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT void JNICALL JFN(destroyContext)(JNIEnv* env, jclass cls, jlong c) {
  (void)env;
  (void)cls;
  rmx_ctx_destroy((rmx_ctx*)(intptr_t)c);
}

/* long createModel(long ctx, int type, long inputDim, int nFields, int embeddingDim, int[] fcDims,
 *                  int[] cinDims, int crossDepth)  -- ctx 0: metadata only (getMatsSize ...) */
JNIEXPORT jlong JNICALL JFN(createModel)(JNIEnv* env, jclass cls, jlong ctx, jint type, jlong input_dim,
                                         jint n_fields, jint k, jintArray fc, jintArray cin, jint cross_depth) {
  (void)cls;
  jsize nfc = fc ? (*env)->GetArrayLength(env, fc) : 0;
  jsize ncin = cin ? (*env)->GetArrayLength(env, cin) : 0;
  jint* pfc = fc ? (*env)->GetIntArrayElements(env, fc, NULL) : NULL;
  jint* pcin = cin ? (*env)->GetIntArrayElements(env, cin, NULL) : NULL;
  rmx_model* m = NULL;
  int st = rmx_model_create((rmx_ctx*)(intptr_t)ctx, type, input_dim, n_fields, k, (const int32_t*)pfc, nfc,
                            (const int32_t*)pcin, ncin, cross_depth, &m);
  if (pfc) (*env)->ReleaseIntArrayElements(env, fc, pfc, JNI_ABORT);
  if (pcin) (*env)->ReleaseIntArrayElements(env, cin, pcin, JNI_ABORT);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  jmodel* j = (jmodel*)calloc(1, sizeof(jmodel));
  if (!j) {
    rmx_model_destroy(m);
    throw_status(env, RMX_E_NOMEM);
    return 0;
  }
  j->m = m;
  j->ctx = (rmx_ctx*)(intptr_t)ctx;
  j->n_fields = n_fields;
  j->k = k;
  pthread_mutex_init(&j->mu, NULL);
  return (jlong)(intptr_t)j;
}

JNIEXPORT void JNICALL JFN(destroyModel)(JNIEnv* env, jclass cls, jlong h) {
  (void)env;
  (void)cls;
  jmodel* j = JM(h);
  if (!j) return;
  rmx_model_destroy(j->m);
  if (j->d_ids) rmx_free(j->ctx, j->d_ids);
  if (j->d_f) rmx_free(j->ctx, j->d_f);
  pthread_mutex_destroy(&j->mu);
  free(j);
}

/* int[] getMatsSize(long model)  -- RecModel.getMatsSize */
JNIEXPORT jintArray JNICALL JFN(getMatsSize)(JNIEnv* env, jclass cls, jlong h) {
  (void)cls;
  int n = 0;
  rmx_model_get_mats_size(JM(h)->m, NULL, 0, &n);
  jintArray out = (*env)->NewIntArray(env, n);
  if (!out || n == 0) return out;
  jint* p = (*env)->GetIntArrayElements(env, out, NULL);
  rmx_model_get_mats_size(JM(h)->m, (int32_t*)p, n, &n);
  (*env)->ReleaseIntArrayElements(env, out, p, 0);
  return out;
}

/* ------------------------------------------------------------------ L-A -- */
/* Critical pointers of the L-A arrays (NULL arrays stay NULL). */
typedef struct {
  jarray a[10];
  void* p[10];
  jint mode[10]; /* 0: copy back (gradients written in place), JNI_ABORT: read-only */
  int n;
} crit;

static void* crit_get(JNIEnv* env, crit* c, jarray a, jint mode) {
  if (!a) return NULL;
  void* p = (*env)->GetPrimitiveArrayCritical(env, a, NULL);
  c->a[c->n] = a;
  c->p[c->n] = p;
  c->mode[c->n] = mode;
  ++c->n;
  return p;
}

static void crit_release(JNIEnv* env, crit* c) {
  while (c->n > 0) {
    --c->n;
    if (c->p[c->n]) (*env)->ReleasePrimitiveArrayCritical(env, c->a[c->n], c->p[c->n], c->mode[c->n]);
  }
}

/* float[] forward0(long model, int batchSize, long[] rows, long[] cols, float[] bias, float[] weights,
 *                  float[] embeddings, int embeddingDim, float[] mats, int[] matSizes, long[] fields)
 * = RecModel.forward(batchSize, batch, bias, weights, embeddings, embeddingDim, mats, matSizes[, fields])
 * with batch = (CooLongFloatMatrix.getRowIndices, getColIndices) (RecModel.scala:146-155). */
JNIEXPORT jfloatArray JNICALL JFN(forward0)(JNIEnv* env, jclass cls, jlong h, jint batch_size, jlongArray rows,
                                            jlongArray cols, jfloatArray bias, jfloatArray weights, jfloatArray emb,
                                            jint k, jfloatArray mats, jintArray mat_sizes, jlongArray fields) {
  (void)cls;
  jfloatArray out = (*env)->NewFloatArray(env, batch_size);
  if (!out) return NULL;
  const jsize nnz = rows ? (*env)->GetArrayLength(env, rows) : 0;
  const jsize nsz = mat_sizes ? (*env)->GetArrayLength(env, mat_sizes) : 0;
  crit c = {{0}, {0}, {0}, 0};
  const int64_t* p_rows = (const int64_t*)crit_get(env, &c, rows, JNI_ABORT);
  const int64_t* p_cols = (const int64_t*)crit_get(env, &c, cols, JNI_ABORT);
  const float* p_bias = (const float*)crit_get(env, &c, bias, JNI_ABORT);
  const float* p_w = (const float*)crit_get(env, &c, weights, JNI_ABORT);
  const float* p_e = (const float*)crit_get(env, &c, emb, JNI_ABORT);
  const float* p_m = (const float*)crit_get(env, &c, mats, JNI_ABORT);
  const int32_t* p_s = (const int32_t*)crit_get(env, &c, mat_sizes, JNI_ABORT);
  const int64_t* p_f = (const int64_t*)crit_get(env, &c, fields, JNI_ABORT);
  float* p_out = (float*)crit_get(env, &c, out, 0);
  const int st = rmx_forward(JM(h)->m, batch_size, nnz, p_rows, p_cols, p_bias, p_w, p_e, k, p_m, p_s, nsz, p_f, p_out);
  crit_release(env, &c);
  if (st) {
    throw_status(env, st);
    return NULL;
  }
  return out;
}

/* float backward0(long model, int batchSize, long[] rows, long[] cols, float[] bias, float[] weights,
 *                 float[] embeddings, int embeddingDim, float[] mats, int[] matSizes, long[] fields,
 *                 float[] targets)
 * = RecModel.backward(...) (RecModel.scala:65-115): bias / weights / embeddings / mats are
 * overwritten IN PLACE with their gradients (util/GradUtil.scala:7-42); returns the mean BCE loss. */
JNIEXPORT jfloat JNICALL JFN(backward0)(JNIEnv* env, jclass cls, jlong h, jint batch_size, jlongArray rows,
                                        jlongArray cols, jfloatArray bias, jfloatArray weights, jfloatArray emb,
                                        jint k, jfloatArray mats, jintArray mat_sizes, jlongArray fields,
                                        jfloatArray targets) {
  (void)cls;
  const jsize nnz = rows ? (*env)->GetArrayLength(env, rows) : 0;
  const jsize nsz = mat_sizes ? (*env)->GetArrayLength(env, mat_sizes) : 0;
  crit c = {{0}, {0}, {0}, 0};
  const int64_t* p_rows = (const int64_t*)crit_get(env, &c, rows, JNI_ABORT);
  const int64_t* p_cols = (const int64_t*)crit_get(env, &c, cols, JNI_ABORT);
  float* p_bias = (float*)crit_get(env, &c, bias, 0);
  float* p_w = (float*)crit_get(env, &c, weights, 0);
  float* p_e = (float*)crit_get(env, &c, emb, 0);
  float* p_m = (float*)crit_get(env, &c, mats, 0);
  const int32_t* p_s = (const int32_t*)crit_get(env, &c, mat_sizes, JNI_ABORT);
  const int64_t* p_f = (const int64_t*)crit_get(env, &c, fields, JNI_ABORT);
  const float* p_t = (const float*)crit_get(env, &c, targets, JNI_ABORT);
  float loss = 0.f;
  const int st =
      rmx_backward(JM(h)->m, batch_size, nnz, p_rows, p_cols, p_bias, p_w, p_e, k, p_m, p_s, nsz, p_f, p_t, &loss);
  crit_release(env, &c);
  if (st) throw_status(env, st);
  return loss;
}

/* ------------------------------------------------------------------ L-B -- */
/* void setMats(long model, float[] mats) / setBias(long model, float bias) / setPrecision(long, int) */
JNIEXPORT void JNICALL JFN(setMats)(JNIEnv* env, jclass cls, jlong h, jfloatArray mats) {
  (void)cls;
  const jsize n = mats ? (*env)->GetArrayLength(env, mats) : 0;
  crit c = {{0}, {0}, {0}, 0};
  const float* p = (const float*)crit_get(env, &c, mats, JNI_ABORT);
  const int st = rmx_model_set_mats(JM(h)->m, p, n);
  crit_release(env, &c);
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL JFN(setBias)(JNIEnv* env, jclass cls, jlong h, jfloat bias) {
  (void)cls;
  const int st = rmx_model_set_bias(JM(h)->m, bias);
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL JFN(setPrecision)(JNIEnv* env, jclass cls, jlong h, jint dtype) {
  (void)cls;
  const int st = rmx_model_set_precision(JM(h)->m, dtype);
  if (st) throw_status(env, st);
}

/* long createTable(long ctx, long rows, int embeddingDim, int dtype) / void destroyTable(long) */
JNIEXPORT jlong JNICALL JFN(createTable)(JNIEnv* env, jclass cls, jlong ctx, jlong rows, jint k, jint dtype) {
  (void)cls;
  rmx_table* t = NULL;
  const int st = rmx_table_create_ex((rmx_ctx*)(intptr_t)ctx, rows, k, dtype, &t);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)t;
}

JNIEXPORT void JNICALL JFN(destroyTable)(JNIEnv* env, jclass cls, jlong t) {
  (void)env;
  (void)cls;
  rmx_table_destroy((rmx_table*)(intptr_t)t);
}

/* void uploadTable(long table, float[] weights, float[] embedding, int layout): the PS rows
 * "weights" / "embedding" (ParRecModel.scala:74-105); layout 0 = the PS's k x V (RMX_LAYOUT_K_MAJOR). */
JNIEXPORT void JNICALL JFN(uploadTable)(JNIEnv* env, jclass cls, jlong t, jfloatArray w, jfloatArray emb,
                                        jint layout) {
  (void)cls;
  const rmx_table* tb = (const rmx_table*)(intptr_t)t;
  const jlong V = rmx_table_rows(tb), kk = rmx_table_embedding_dim(tb);
  if (!require_arg(env, V >= 0 && (!w || alen(env, w) == V), "uploadTable: weights must hold the table's rows") ||
      !require_arg(env, !emb || alen(env, emb) == V * kk,
                   "uploadTable: embedding must hold rows * embeddingDim floats"))
    return;
  crit c = {{0}, {0}, {0}, 0};
  const float* pw = (const float*)crit_get(env, &c, w, JNI_ABORT);
  const float* pe = (const float*)crit_get(env, &c, emb, JNI_ABORT);
  const int st = rmx_table_upload((rmx_table*)(intptr_t)t, pw, pe, layout);
  crit_release(env, &c);
  if (st) throw_status(env, st);
}

JNIEXPORT void JNICALL JFN(fillTableSynthetic)(JNIEnv* env, jclass cls, jlong t, jlong seed) {
  (void)cls;
  const int st = rmx_table_fill_synthetic((rmx_table*)(intptr_t)t, (uint64_t)seed);
  if (st) throw_status(env, st);
}

/* Stage the int32 ids [n] of a batch on the device (the model's staging buffer). */
static int stage_ids(JNIEnv* env, jmodel* j, jintArray ids, size_t n) {
  int st = grow(j->ctx, &j->d_ids, &j->cap_ids, n ? n : 1, sizeof(int32_t));
  if (st || n == 0) return st;
  void* p = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
  st = rmx_memcpy_htod(j->ctx, j->d_ids, p, n * sizeof(int32_t));
  (*env)->ReleasePrimitiveArrayCritical(env, ids, p, JNI_ABORT);
  return st;
}

/* Copy n floats at device offset off of the float staging into a new (or the given) Java array. */
static int unstage(JNIEnv* env, jmodel* j, size_t off, size_t n, jfloatArray dst) {
  if (n == 0) return RMX_OK;
  void* p = (*env)->GetPrimitiveArrayCritical(env, dst, NULL);
  const int st = rmx_memcpy_dtoh(j->ctx, p, (float*)j->d_f + off, n * sizeof(float));
  (*env)->ReleasePrimitiveArrayCritical(env, dst, p, 0);
  return st;
}

/* float[] forwardIds(long model, long table, int batch, int[] ids)  -- ids [batch * nFields], the
 * COO column indices in field order (SampleParser id - 1).  pull + make* + forward in one call
 * (ParRecModel.predictBiasWeightEmbeddingMats, ParRecModel.scala:555-567). */
JNIEXPORT jfloatArray JNICALL JFN(forwardIds)(JNIEnv* env, jclass cls, jlong h, jlong t, jint batch, jintArray ids) {
  (void)cls;
  jmodel* j = JM(h);
  if (!require_arg(env, batch >= 0 && alen(env, ids) == (jlong)batch * j->n_fields,
                   "forwardIds: ids must hold batch * nFields ints"))
    return NULL;
  const jsize n = (*env)->GetArrayLength(env, ids);
  jfloatArray out = (*env)->NewFloatArray(env, batch);
  if (!out) return NULL;
  pthread_mutex_lock(&j->mu);
  int st = stage_ids(env, j, ids, (size_t)n);
  if (!st) st = grow(j->ctx, &j->d_f, &j->cap_f, batch > 0 ? batch : 1, sizeof(float));
  if (!st) st = rmx_forward_ids(j->m, (rmx_table*)(intptr_t)t, batch, (const int32_t*)j->d_ids, (float*)j->d_f, NULL);
  if (!st) st = unstage(env, j, 0, (size_t)batch, out);
  pthread_mutex_unlock(&j->mu);
  if (st) {
    throw_status(env, st);
    return NULL;
  }
  return out;
}

/* float[] predictIds(long model, long table, long nRows, int[] ids, int batch)
 * -- ParRecModel.predict over a row set (ParRecModel.scala:519-581), `batch` rows per forward. */
JNIEXPORT jfloatArray JNICALL JFN(predictIds)(JNIEnv* env, jclass cls, jlong h, jlong t, jlong n_rows, jintArray ids,
                                              jint batch) {
  (void)cls;
  jmodel* j = JM(h);
  if (!require_arg(env, n_rows >= 0 && n_rows <= 0x7fffffff && batch > 0 &&
                            alen(env, ids) == n_rows * (jlong)j->n_fields,
                   "predictIds: need nRows >= 0, batch > 0 and ids of nRows * nFields ints"))
    return NULL;
  const jsize n = (*env)->GetArrayLength(env, ids);
  jfloatArray out = (*env)->NewFloatArray(env, (jsize)n_rows);
  if (!out) return NULL;
  pthread_mutex_lock(&j->mu);
  int st = stage_ids(env, j, ids, (size_t)n);
  if (!st) st = grow(j->ctx, &j->d_f, &j->cap_f, n_rows > 0 ? (size_t)n_rows : 1, sizeof(float));
  if (!st)
    st = rmx_predict_ids(j->m, (rmx_table*)(intptr_t)t, n_rows, (const int32_t*)j->d_ids, batch, (float*)j->d_f, NULL);
  if (!st) st = unstage(env, j, 0, (size_t)n_rows, out);
  pthread_mutex_unlock(&j->mu);
  if (st) {
    throw_status(env, st);
    return NULL;
  }
  return out;
}

/* float backwardIds(long model, long table, int batch, int[] ids, float[] targets, float[] gBias,
 *                   float[] gWeights, float[] gEmbedding, float[] gMats)
 * One training pass over ids [batch * nFields] on the HBM table: the gradient arrays (each may be
 * null) receive what RecModel.backward writes back -- gBias [1], gWeights [batch*F] and gEmbedding
 * [batch*F*k] per nonzero (what makeGrad / push take, ParRecModel.scala:439-478), gMats [matsLen];
 * returns the mean BCE loss. */
JNIEXPORT jfloat JNICALL JFN(backwardIds)(JNIEnv* env, jclass cls, jlong h, jlong t, jint batch, jintArray ids,
                                          jfloatArray targets, jfloatArray g_bias, jfloatArray g_w, jfloatArray g_e,
                                          jfloatArray g_m) {
  (void)cls;
  jmodel* j = JM(h);
  const jlong nnz = (jlong)batch * j->n_fields;
  const int64_t ml = rmx_model_mats_len(j->m);
  if (!require_arg(env, batch >= 0 && alen(env, ids) == nnz, "backwardIds: ids must hold batch * nFields ints") ||
      !require_arg(env, alen(env, targets) >= batch, "backwardIds: targets must hold batch floats") ||
      !require_arg(env, !g_bias || alen(env, g_bias) >= 1, "backwardIds: gBias must hold 1 float") ||
      !require_arg(env, !g_w || alen(env, g_w) == nnz, "backwardIds: gWeights must hold batch * nFields floats") ||
      !require_arg(env, !g_e || alen(env, g_e) == nnz * j->k,
                   "backwardIds: gEmbedding must hold batch * nFields * embeddingDim floats") ||
      !require_arg(env, !g_m || alen(env, g_m) == ml, "backwardIds: gMats must hold the model's mats length"))
    return 0.f;
  const jsize n = (*env)->GetArrayLength(env, ids);
  const size_t nb = (size_t)batch, ng = g_w ? (size_t)(*env)->GetArrayLength(env, g_w) : 0,
               ne = g_e ? (size_t)(*env)->GetArrayLength(env, g_e) : 0,
               nm = g_m ? (size_t)(*env)->GetArrayLength(env, g_m) : 0;
  /* float staging: [targets B][loss 1][g_bias 1][g_w][g_e][g_m] */
  const size_t o_t = 0, o_l = nb, o_b = nb + 1, o_w = nb + 2, o_e = o_w + ng, o_m = o_e + ne, tot = o_m + nm;
  float loss = 0.f;
  pthread_mutex_lock(&j->mu);
  int st = stage_ids(env, j, ids, (size_t)n);
  if (!st) st = grow(j->ctx, &j->d_f, &j->cap_f, tot, sizeof(float));
  if (!st && nb) {
    void* p = (*env)->GetPrimitiveArrayCritical(env, targets, NULL);
    st = rmx_memcpy_htod(j->ctx, (float*)j->d_f + o_t, p, nb * sizeof(float));
    (*env)->ReleasePrimitiveArrayCritical(env, targets, p, JNI_ABORT);
  }
  float* f = (float*)j->d_f;
  if (!st)
    st = rmx_backward_ids(j->m, (rmx_table*)(intptr_t)t, batch, (const int32_t*)j->d_ids, f + o_t,
                          g_bias ? f + o_b : NULL, g_w ? f + o_w : NULL, g_e ? f + o_e : NULL, g_m ? f + o_m : NULL,
                          f + o_l, NULL);
  if (!st) st = rmx_memcpy_dtoh(j->ctx, &loss, f + o_l, sizeof(float));
  if (!st && g_bias) st = unstage(env, j, o_b, 1, g_bias);
  if (!st && g_w) st = unstage(env, j, o_w, ng, g_w);
  if (!st && g_e) st = unstage(env, j, o_e, ne, g_e);
  if (!st && g_m) st = unstage(env, j, o_m, nm, g_m);
  pthread_mutex_unlock(&j->mu);
  if (st) throw_status(env, st);
  return loss;
}

/* double auc(long model, float[] labels, float[] scores)  -- the examples' per-epoch metric
 * (example/DeepFMLocalExample.scala:44-52), on the model's device. */
JNIEXPORT jdouble JNICALL JFN(auc)(JNIEnv* env, jclass cls, jlong h, jfloatArray labels, jfloatArray scores) {
  (void)cls;
  jmodel* j = JM(h);
  if (!require_arg(env, labels && scores && alen(env, labels) == alen(env, scores),
                   "auc: labels and scores must be arrays of the same length"))
    return 0.0;
  const jsize n = (*env)->GetArrayLength(env, labels);
  double a = 0.0;
  pthread_mutex_lock(&j->mu);
  int st = grow(j->ctx, &j->d_f, &j->cap_f, 2 * (size_t)(n > 0 ? n : 1), sizeof(float));
  float* f = (float*)j->d_f;
  for (int i = 0; i < 2 && !st && n > 0; ++i) {
    jfloatArray src = i == 0 ? labels : scores;
    void* p = (*env)->GetPrimitiveArrayCritical(env, src, NULL);
    st = rmx_memcpy_htod(j->ctx, f + (size_t)i * n, p, (size_t)n * sizeof(float));
    (*env)->ReleasePrimitiveArrayCritical(env, src, p, JNI_ABORT);
  }
  if (!st) st = rmx_auc(j->ctx, n, f, f + n, &a, NULL);
  pthread_mutex_unlock(&j->mu);
  if (st) throw_status(env, st);
  return a;
}

/* ---------------------------------------------------------- sharded table -- */
/* byte[] commUniqueId()  -- rank 0 creates it, the driver broadcasts it (e.g. a Spark broadcast) */
JNIEXPORT jbyteArray JNICALL JFN(commUniqueId)(JNIEnv* env, jclass cls) {
  (void)cls;
  char buf[RMX_UNIQUE_ID_BYTES];
  const int st = rmx_comm_unique_id(buf, sizeof(buf));
  if (st) {
    throw_status(env, st);
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, RMX_UNIQUE_ID_BYTES);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, RMX_UNIQUE_ID_BYTES, (const jbyte*)buf);
  return out;
}

/* long createShard(long ctx, long rows, int embeddingDim, int nranks, int rank, byte[] uniqueId) */
JNIEXPORT jlong JNICALL JFN(createShard)(JNIEnv* env, jclass cls, jlong ctx, jlong rows, jint k, jint nranks,
                                         jint rank, jbyteArray uid) {
  (void)cls;
  char buf[RMX_UNIQUE_ID_BYTES];
  if (!uid || (*env)->GetArrayLength(env, uid) != RMX_UNIQUE_ID_BYTES) {
    jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (c) (*env)->ThrowNew(env, c, "createShard: uniqueId must hold RMX_UNIQUE_ID_BYTES bytes");
    return 0;
  }
  (*env)->GetByteArrayRegion(env, uid, 0, RMX_UNIQUE_ID_BYTES, (jbyte*)buf);
  rmx_shard* sh = NULL;
  const int st = rmx_shard_create((rmx_ctx*)(intptr_t)ctx, rows, k, nranks, rank, buf, &sh);
  if (st) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)sh;
}

JNIEXPORT void JNICALL JFN(destroyShard)(JNIEnv* env, jclass cls, jlong sh) {
  (void)env;
  (void)cls;
  rmx_shard_destroy((rmx_shard*)(intptr_t)sh);
}

JNIEXPORT void JNICALL JFN(fillShardSynthetic)(JNIEnv* env, jclass cls, jlong sh, jlong seed) {
  (void)cls;
  const int st = rmx_shard_fill_synthetic((rmx_shard*)(intptr_t)sh, (uint64_t)seed);
  if (st) throw_status(env, st);
}

/* void setShardOwnerHash(long shard, long key) -- before fillShardSynthetic, the same key on every rank */
JNIEXPORT void JNICALL JFN(setShardOwnerHash)(JNIEnv* env, jclass cls, jlong sh, jlong key) {
  (void)cls;
  const int st = rmx_shard_set_owner_hash((rmx_shard*)(intptr_t)sh, (uint64_t)key);
  if (st) throw_status(env, st);
}

/* float[] forwardIdsSharded(long model, long shard, int batch, int[] ids)  -- collective: every rank
 * calls it with its own batch (the exchange replaces the PS pulls, ParRecModel.scala:165-199). */
JNIEXPORT jfloatArray JNICALL JFN(forwardIdsSharded)(JNIEnv* env, jclass cls, jlong h, jlong sh, jint batch,
                                                     jintArray ids) {
  (void)cls;
  jmodel* j = JM(h);
  if (!require_arg(env, batch >= 0 && alen(env, ids) == (jlong)batch * j->n_fields,
                   "forwardIdsSharded: ids must hold batch * nFields ints"))
    return NULL;
  const jsize n = (*env)->GetArrayLength(env, ids);
  jfloatArray out = (*env)->NewFloatArray(env, batch);
  if (!out) return NULL;
  pthread_mutex_lock(&j->mu);
  int st = stage_ids(env, j, ids, (size_t)n);
  if (!st) st = grow(j->ctx, &j->d_f, &j->cap_f, batch > 0 ? batch : 1, sizeof(float));
  if (!st)
    st = rmx_forward_ids_sharded(j->m, (rmx_shard*)(intptr_t)sh, batch, (const int32_t*)j->d_ids, (float*)j->d_f,
                                 NULL);
  if (!st) st = unstage(env, j, 0, (size_t)batch, out);
  pthread_mutex_unlock(&j->mu);
  if (st) {
    throw_status(env, st);
    return NULL;
  }
  return out;
}

#else
/* No <jni.h> in this toolchain: nothing to build (the C ABI in librmx.so is the boundary). */
typedef int rmx_jni_unavailable;
#endif
