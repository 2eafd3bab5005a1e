/*
 * rmx_jni.c -- thin JNI shim from the reference's Scala RecModel plugin API to librmx.so.
 *
 * The reference calls `RecModel.forward(batchSize, batch, bias, weights, embeddings,
 * embeddingDim, mats, matSizes)` (src/main/scala/io/yaochi/recommendation/model/RecModel.scala:37-48)
 * from ParRecModel.predict / optimize (model/ParRecModel.scala:365-581).  A Scala class
 * `io.yaochi.recommendation.model.gpu.GpuRecModel` declares the natives below;
 * each one pins the JVM arrays (GetPrimitiveArrayCritical, no copy on HotSpot) and calls the
 * C ABI of include/rmx.h.  Errors become Java exceptions with the reference's types:
 *   RMX_E_INDEX / RMX_E_INVALID -> IllegalArgumentException   (bnn/Scatter.scala:29-30 require)
 *   RMX_E_SHAPE / RMX_E_MATS    -> IllegalArgumentException   (BigDL Reshape size mismatch)
 *   RMX_E_TYPE                  -> scala.MatchError is not reachable from C: IllegalStateException
 *   RMX_E_HIP / RMX_E_NOMEM     -> RuntimeException
 *
 * Build (needs a JDK; this container and the GPU box have none, so it is not built here):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *      rmx_jni.c -L../csrc -lrmx -Wl,-rpath,'$ORIGIN' -o librmx_jni.so
 */
#if defined(__has_include)
#if __has_include(<jni.h>)
#define RMX_HAVE_JNI 1
#endif
#endif

#ifdef RMX_HAVE_JNI
#include <jni.h>
#include <stdint.h>

#include "../../include/rmx.h"

static void throw_status(JNIEnv* env, int st) {
  const char* cls = "java/lang/RuntimeException";
  if (st == RMX_E_INDEX || st == RMX_E_INVALID || st == RMX_E_SHAPE || st == RMX_E_MATS)
    cls = "java/lang/IllegalArgumentException";
  else if (st == RMX_E_TYPE)
    cls = "java/lang/IllegalStateException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, rmx_last_error());
}

/* long createModel(int type, long inputDim, int nFields, int embeddingDim, int[] fcDims,
 *                  int[] cinDims, int crossDepth, int device)  -- device < 0: metadata only */
JNIEXPORT jlong JNICALL Java_io_yaochi_recommendation_model_gpu_GpuRecModel_createModel(
    JNIEnv* env, jclass cls, jint type, jlong input_dim, jint n_fields, jint k, jintArray fc, jintArray cin,
    jint cross_depth, jint device) {
  (void)cls;
  rmx_ctx* ctx = NULL;
  if (device >= 0) {
    int st = rmx_ctx_create(device, &ctx);
    if (st) { throw_status(env, st); return 0; }
  }
  jsize nfc = fc ? (*env)->GetArrayLength(env, fc) : 0;
  jsize ncin = cin ? (*env)->GetArrayLength(env, cin) : 0;
  jint* pfc = fc ? (*env)->GetIntArrayElements(env, fc, NULL) : NULL;
  jint* pcin = cin ? (*env)->GetIntArrayElements(env, cin, NULL) : NULL;
  rmx_model* m = NULL;
  int st = rmx_model_create(ctx, type, input_dim, n_fields, k, (const int32_t*)pfc, nfc, (const int32_t*)pcin,
                            ncin, cross_depth, &m);
  if (pfc) (*env)->ReleaseIntArrayElements(env, fc, pfc, JNI_ABORT);
  if (pcin) (*env)->ReleaseIntArrayElements(env, cin, pcin, JNI_ABORT);
  if (st) { throw_status(env, st); return 0; }
  return (jlong)(intptr_t)m;
}

JNIEXPORT void JNICALL Java_io_yaochi_recommendation_model_gpu_GpuRecModel_destroyModel(JNIEnv* env, jclass cls,
                                                                                      jlong h) {
  (void)env;
  (void)cls;
  rmx_model_destroy((rmx_model*)(intptr_t)h);
}

/* int[] getMatsSize(long model)  -- RecModel.getMatsSize */
JNIEXPORT jintArray JNICALL Java_io_yaochi_recommendation_model_gpu_GpuRecModel_getMatsSize(JNIEnv* env, jclass cls,
                                                                                          jlong h) {
  (void)cls;
  int n = 0;
  rmx_model_get_mats_size((rmx_model*)(intptr_t)h, NULL, 0, &n);
  jintArray out = (*env)->NewIntArray(env, n);
  if (!out || n == 0) return out;
  jint* p = (*env)->GetIntArrayElements(env, out, NULL);
  rmx_model_get_mats_size((rmx_model*)(intptr_t)h, (int32_t*)p, n, &n);
  (*env)->ReleaseIntArrayElements(env, out, p, 0);
  return out;
}

/* float[] forward0(long model, int batchSize, long[] rows, long[] cols, float[] bias, float[] weights,
 *                  float[] embeddings, int embeddingDim, float[] mats, int[] matSizes)
 * = RecModel.forward(batchSize, batch, bias, weights, embeddings, embeddingDim, mats, matSizes)
 * with batch = (CooLongFloatMatrix.getRowIndices, getColIndices) (RecModel.scala:146-155). */
JNIEXPORT jfloatArray JNICALL Java_io_yaochi_recommendation_model_gpu_GpuRecModel_forward0(
    JNIEnv* env, jclass cls, jlong h, jint batch_size, jlongArray rows, jlongArray cols, jfloatArray bias,
    jfloatArray weights, jfloatArray emb, jint k, jfloatArray mats, jintArray mat_sizes) {
  (void)cls;
  jfloatArray out = (*env)->NewFloatArray(env, batch_size);
  if (!out) return NULL;
  const jsize nnz = rows ? (*env)->GetArrayLength(env, rows) : 0;
  const jsize nsz = mat_sizes ? (*env)->GetArrayLength(env, mat_sizes) : 0;
  /* Critical sections must not call back into the JVM: take every pointer, call, release. */
  void* p_rows = rows ? (*env)->GetPrimitiveArrayCritical(env, rows, NULL) : NULL;
  void* p_cols = cols ? (*env)->GetPrimitiveArrayCritical(env, cols, NULL) : NULL;
  void* p_bias = bias ? (*env)->GetPrimitiveArrayCritical(env, bias, NULL) : NULL;
  void* p_w = weights ? (*env)->GetPrimitiveArrayCritical(env, weights, NULL) : NULL;
  void* p_e = emb ? (*env)->GetPrimitiveArrayCritical(env, emb, NULL) : NULL;
  void* p_m = mats ? (*env)->GetPrimitiveArrayCritical(env, mats, NULL) : NULL;
  void* p_s = mat_sizes ? (*env)->GetPrimitiveArrayCritical(env, mat_sizes, NULL) : NULL;
  void* p_out = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  const int st = rmx_forward((rmx_model*)(intptr_t)h, batch_size, nnz, (const int64_t*)p_rows,
                             (const int64_t*)p_cols, (const float*)p_bias, (const float*)p_w, (const float*)p_e, k,
                             (const float*)p_m, (const int32_t*)p_s, nsz, NULL, (float*)p_out);
  (*env)->ReleasePrimitiveArrayCritical(env, out, p_out, 0);
  if (p_s) (*env)->ReleasePrimitiveArrayCritical(env, mat_sizes, p_s, JNI_ABORT);
  if (p_m) (*env)->ReleasePrimitiveArrayCritical(env, mats, p_m, JNI_ABORT);
  if (p_e) (*env)->ReleasePrimitiveArrayCritical(env, emb, p_e, JNI_ABORT);
  if (p_w) (*env)->ReleasePrimitiveArrayCritical(env, weights, p_w, JNI_ABORT);
  if (p_bias) (*env)->ReleasePrimitiveArrayCritical(env, bias, p_bias, JNI_ABORT);
  if (p_cols) (*env)->ReleasePrimitiveArrayCritical(env, cols, p_cols, JNI_ABORT);
  if (p_rows) (*env)->ReleasePrimitiveArrayCritical(env, rows, p_rows, JNI_ABORT);
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
