/* JNI glue for sparky.hip.PageRankJni (JDK 8..21 hosts): copies the Java arrays, calls the C ABI
 * of include/pagerank_hip.h and forwards every iteration to the Java listener.  The arrays are
 * borrowed for the call only, as the ABI specifies.  Build: java/Makefile (needs a JDK's jni.h). */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pagerank_hip.h"

typedef struct {
  JNIEnv *env;
  jobject listener;
  jmethodID on_iter;
  int32_t n;
  int failed;
} cb_ctx;

static void on_iter(int32_t it, const double *ranks, double dc, double l1, double ms, void *user) {
  cb_ctx *c = (cb_ctx *)user;
  JNIEnv *env = c->env;
  if (!c->listener || c->failed) return;
  jdoubleArray r = NULL;
  if (ranks) {
    r = (*env)->NewDoubleArray(env, c->n);
    if (!r) { c->failed = 1; return; }
    (*env)->SetDoubleArrayRegion(env, r, 0, c->n, ranks);
  }
  (*env)->CallVoidMethod(env, c->listener, c->on_iter, (jint)it, r, dc, l1, ms);
  if ((*env)->ExceptionCheck(env)) c->failed = 1; /* rethrown when run returns */
  if (r) (*env)->DeleteLocalRef(env, r);
}

static jdoubleArray fail(JNIEnv *env, int rc) {
  char msg[1024];
  snprintf(msg, sizeof(msg), "libpagerank_hip error %d: %s", rc, pr_last_error());
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  if (ex) (*env)->ThrowNew(env, ex, msg);
  return NULL;
}

JNIEXPORT jint JNICALL Java_sparky_hip_PageRankJni_abiVersion(JNIEnv *env, jclass cls) {
  (void)env;
  (void)cls;
  return (jint)pr_abi_version();
}

JNIEXPORT jdoubleArray JNICALL Java_sparky_hip_PageRankJni_run(JNIEnv *env, jclass cls, jint device, jint n_vertices,
                                                               jintArray jsrc, jintArray jdst, jint flags,
                                                               jint iterations, jdoubleArray jinit, jobject listener,
                                                               jboolean ranks_in_cb) {
  (void)cls;
  const jsize E = (*env)->GetArrayLength(env, jsrc);
  if ((*env)->GetArrayLength(env, jdst) != E) return fail(env, PR_ERR_INVALID);
  if (jinit && (*env)->GetArrayLength(env, jinit) != n_vertices) return fail(env, PR_ERR_INVALID);
  /* Get*ArrayElements / malloc return NULL on OOM (an OutOfMemoryError is then pending for the
   * JNI calls): release what was obtained and return */
  jint *src = (*env)->GetIntArrayElements(env, jsrc, NULL);
  if (!src) return NULL;
  jint *dst = (*env)->GetIntArrayElements(env, jdst, NULL);
  if (!dst) {
    (*env)->ReleaseIntArrayElements(env, jsrc, src, JNI_ABORT);
    return NULL;
  }
  pr_graph *g = NULL;
  int rc = pr_graph_create(device, n_vertices, (int64_t)E, (const int32_t *)src, (const int32_t *)dst,
                           (uint32_t)flags | PR_NO_CANONICAL, &g);
  (*env)->ReleaseIntArrayElements(env, jsrc, src, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, jdst, dst, JNI_ABORT);
  if (rc != PR_OK) return fail(env, rc);
  double *init = NULL;
  if (jinit) {
    init = (double *)(*env)->GetDoubleArrayElements(env, jinit, NULL);
    if (!init) {
      pr_graph_destroy(g);
      return NULL;
    }
  }
  double *ranks = (double *)malloc(sizeof(double) * (size_t)(n_vertices > 0 ? n_vertices : 1));
  if (!ranks) {
    if (jinit) (*env)->ReleaseDoubleArrayElements(env, jinit, (jdouble *)init, JNI_ABORT);
    pr_graph_destroy(g);
    return fail(env, PR_ERR_OOM);
  }
  cb_ctx ctx = {env, listener, NULL, n_vertices, 0};
  if (listener) {
    jclass lc = (*env)->GetObjectClass(env, listener);
    ctx.on_iter = (*env)->GetMethodID(env, lc, "onIteration", "(I[DDDD)V");
  }
  rc = pr_run(g, iterations, 0.15, 0.85, init, ranks, listener ? on_iter : NULL, ranks_in_cb ? PR_CB_RANKS : 0u, &ctx);
  if (jinit) (*env)->ReleaseDoubleArrayElements(env, jinit, (jdouble *)init, JNI_ABORT);
  pr_graph_destroy(g);
  if (ctx.failed || (*env)->ExceptionCheck(env)) {
    free(ranks);
    return NULL; /* the listener's exception propagates */
  }
  if (rc != PR_OK) {
    free(ranks);
    return fail(env, rc);
  }
  jdoubleArray out = (*env)->NewDoubleArray(env, n_vertices);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, n_vertices, ranks);
  free(ranks);
  return out;
}
