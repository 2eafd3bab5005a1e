/*
 * fake_jni.c -- TEST HARNESS ONLY: an in-process stand-in for the JVM side of the JNI calls that
 * recommendation-models_amd/jni/rmx_jni.c makes (arrays, exceptions), so tests/test_jni_shim.py
 * can call the shim's natives from Python (ctypes) exactly as Scala would call them, and compare
 * them with librmx's C ABI.  Java arrays are {kind, length, data}; Get*Critical returns the data
 * (no copy, like HotSpot); the release mode is recorded so a test can check that gradients are
 * written back (mode 0) and inputs are not (JNI_ABORT).
 */
#include <stdlib.h>
#include <string.h>

#include <jni.h>

struct fake_obj {
  int kind; /* 0 class, 1 int[], 2 long[], 3 float[], 4 byte[] */
  jsize n;
  void* data;
  char name[96];
  int last_release_mode;
};

static char g_exc_class[96], g_exc_msg[512];
static int g_exc = 0;

static size_t esize(int kind) { return kind == 2 ? 8 : kind == 4 ? 1 : 4; }

static jobject new_arr(int kind, jsize n) {
  jobject a = (jobject)calloc(1, sizeof(struct fake_obj));
  a->kind = kind;
  a->n = n;
  a->data = calloc(n > 0 ? (size_t)n : 1, esize(kind));
  a->last_release_mode = -1;
  return a;
}

static jclass f_find_class(JNIEnv* e, const char* name) {
  (void)e;
  jclass c = (jclass)calloc(1, sizeof(struct fake_obj));
  strncpy(c->name, name, sizeof(c->name) - 1);
  return c; /* leaked: a test-only handful */
}
static jint f_throw_new(JNIEnv* e, jclass c, const char* msg) {
  (void)e;
  g_exc = 1;
  strncpy(g_exc_class, c->name, sizeof(g_exc_class) - 1);
  strncpy(g_exc_msg, msg ? msg : "", sizeof(g_exc_msg) - 1);
  return 0;
}
static jsize f_len(JNIEnv* e, jarray a) { (void)e; return a->n; }
static jint* f_get_ints(JNIEnv* e, jintArray a, jboolean* c) { (void)e; if (c) *c = 0; return (jint*)a->data; }
static void f_rel_ints(JNIEnv* e, jintArray a, jint* p, jint mode) { (void)e; (void)p; a->last_release_mode = mode; }
static void* f_get_crit(JNIEnv* e, jarray a, jboolean* c) { (void)e; if (c) *c = 0; return a->data; }
static void f_rel_crit(JNIEnv* e, jarray a, void* p, jint mode) { (void)e; (void)p; a->last_release_mode = mode; }
static jintArray f_new_int(JNIEnv* e, jsize n) { (void)e; return new_arr(1, n); }
static jfloatArray f_new_float(JNIEnv* e, jsize n) { (void)e; return new_arr(3, n); }
static jbyteArray f_new_byte(JNIEnv* e, jsize n) { (void)e; return new_arr(4, n); }
static void f_get_bytes(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* b) { (void)e; memcpy(b, (jbyte*)a->data + s, n); }
static void f_set_bytes(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* b) { (void)e; memcpy((jbyte*)a->data + s, b, n); }

static const struct JNINativeInterface_ g_table = {f_find_class, f_throw_new, f_len, f_get_ints, f_rel_ints,
                                                   f_get_crit, f_rel_crit, f_new_int, f_new_float, f_new_byte,
                                                   f_get_bytes, f_set_bytes};
static JNIEnv g_env = &g_table;

/* ---- ctypes helpers ---- */
JNIEnv* fj_env(void) { return &g_env; }
jobject fj_new_array(int kind, jsize n, const void* src) {
  jobject a = new_arr(kind, n);
  if (src && n > 0) memcpy(a->data, src, (size_t)n * esize(kind));
  return a;
}
void* fj_data(jobject a) { return a ? a->data : NULL; }
jsize fj_len(jobject a) { return a ? a->n : -1; }
int fj_release_mode(jobject a) { return a ? a->last_release_mode : -1; }
void fj_free(jobject a) {
  if (!a) return;
  free(a->data);
  free(a);
}
/* last thrown exception: class name and message ("" when none); fj_clear resets */
int fj_exception(char* cls, int ccap, char* msg, int mcap) {
  if (!g_exc) return 0;
  strncpy(cls, g_exc_class, ccap - 1);
  cls[ccap - 1] = 0;
  strncpy(msg, g_exc_msg, mcap - 1);
  msg[mcap - 1] = 0;
  return 1;
}
void fj_clear(void) { g_exc = 0; }
