/*
 * mock_env.c — test infrastructure only (tests/test_jni_shim.py): runs jni/stcjni.c's wrappers against
 * a mock JNIEnv (arrays are host buffers with a length; ThrowNew records the exception) and the real
 * libstc.so, with no JVM and no GPU.  Each case prints one line: name, thrown class, message.
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../jni/stcjni.c"

struct _jobject {
  const char* name; /* classes */
  jsize len;        /* arrays */
  void* data;
};
static char g_cls[128], g_msg[512];
static int g_thrown;

static jclass m_FindClass(JNIEnv* e, const char* name) {
  jclass c = calloc(1, sizeof *c);
  c->name = name;
  return c;
}
static jint m_ThrowNew(JNIEnv* e, jclass c, const char* msg) {
  snprintf(g_cls, sizeof g_cls, "%s", c->name);
  snprintf(g_msg, sizeof g_msg, "%s", msg);
  g_thrown = 1;
  return 0;
}
static jboolean m_ExceptionCheck(JNIEnv* e) { return (jboolean)g_thrown; }
static jsize m_GetArrayLength(JNIEnv* e, jarray a) { return a->len; }
static jstring m_NewStringUTF(JNIEnv* e, const char* s) { return NULL; }
static jarray new_array(jsize n, size_t esz) {
  jarray a = calloc(1, sizeof *a);
  a->len = n;
  a->data = calloc(n > 0 ? (size_t)n : 1, esz);
  return a;
}
static jbyteArray m_NewByteArray(JNIEnv* e, jsize n) { return new_array(n, 1); }
static jlongArray m_NewLongArray(JNIEnv* e, jsize n) { return new_array(n, 8); }
static jdoubleArray m_NewDoubleArray(JNIEnv* e, jsize n) { return new_array(n, 8); }
static jbyte* m_GetB(JNIEnv* e, jbyteArray a, jboolean* c) { return a->data; }
static jint* m_GetI(JNIEnv* e, jintArray a, jboolean* c) { return a->data; }
static jlong* m_GetL(JNIEnv* e, jlongArray a, jboolean* c) { return a->data; }
static jdouble* m_GetD(JNIEnv* e, jdoubleArray a, jboolean* c) { return a->data; }
static void m_RelB(JNIEnv* e, jbyteArray a, jbyte* p, jint m) {}
static void m_RelI(JNIEnv* e, jintArray a, jint* p, jint m) {}
static void m_RelL(JNIEnv* e, jlongArray a, jlong* p, jint m) {}
static void m_RelD(JNIEnv* e, jdoubleArray a, jdouble* p, jint m) {}
static void m_GetBR(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* o) { memcpy(o, (jbyte*)a->data + s, n); }
static void m_GetLR(JNIEnv* e, jlongArray a, jsize s, jsize n, jlong* o) { memcpy(o, (jlong*)a->data + s, 8 * n); }
static void m_SetBR(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* i) { memcpy((jbyte*)a->data + s, i, n); }
static void m_SetLR(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* i) { memcpy((jlong*)a->data + s, i, 8 * n); }
static void m_SetDR(JNIEnv* e, jdoubleArray a, jsize s, jsize n, const jdouble* i) {
  memcpy((jdouble*)a->data + s, i, 8 * n);
}

static const struct JNINativeInterface_ table = {
    m_FindClass, m_ThrowNew, m_ExceptionCheck, m_GetArrayLength, m_NewStringUTF, m_NewByteArray,
    m_NewLongArray, m_NewDoubleArray, m_GetB, m_GetI, m_GetL, m_GetD, m_RelB, m_RelI, m_RelL, m_RelD,
    m_GetBR, m_GetLR, m_SetBR, m_SetLR, m_SetDR};

static void report(const char* name) {
  printf("%s\t%s\t%s\n", name, g_thrown ? g_cls : "-", g_thrown ? g_msg : "-");
  g_thrown = 0;
  g_cls[0] = g_msg[0] = 0;
}
static jarray arr(jsize n, size_t esz) { return new_array(n, esz); }

/* GPU mode (tests/test_gpu_jni_shim.py): a real context, IDF model and group behind the same wrappers */
static int gpu_main(JNIEnv* env) {
  jlong ctx = FN(init)(env, NULL, 0);
  report("init");
  if (!ctx) return 1;
  /* 3 documents over 10 terms: {0:2, 3:1}, {3:4}, {1:1, 3:2, 9:5} */
  jlongArray ip = arr(4, 8);
  jintArray ix = arr(6, 4);
  jdoubleArray vs = arr(6, 8);
  jlong p4[4] = {0, 2, 3, 6};
  jint i6[6] = {0, 3, 3, 1, 3, 9};
  jdouble v6[6] = {2, 1, 4, 1, 2, 5};
  memcpy(ip->data, p4, sizeof p4);
  memcpy(ix->data, i6, sizeof i6);
  memcpy(vs->data, v6, sizeof v6);
  jlong m = FN(dcsrUpload)(env, NULL, ctx, 3, 10, ip, ix, vs, 1);
  report("dcsrUpload");
  jlong model = FN(idfFitDev)(env, NULL, ctx, m, 0);
  report("idfFitDev");
  FN(idfGet)(env, NULL, ctx, model, 9, arr(10, 8), NULL);
  report("idfGet_wrong_cols");     /* the model has 10 columns */
  FN(idfGet)(env, NULL, ctx, model, 10, arr(9, 8), NULL);
  report("idfGet_short_idf");
  {
    jlongArray df = arr(10, 8);
    jlong mm = FN(idfGet)(env, NULL, ctx, model, 10, arr(10, 8), df);
    report("idfGet_sized");
    const jlong* d = df->data;
    printf("idfGet_result\t%lld\t%lld %lld %lld %lld\n", (long long)mm, (long long)d[0], (long long)d[1],
           (long long)d[3], (long long)d[9]);
  }
  FN(didfFree)(env, NULL, model);
  FN(dcsrFree)(env, NULL, m);
  /* HipLDAModel.transform's call: a one-device group, λ set, θ of the 3 documents */
  jintArray dev = arr(1, 4);
  jlong g = FN(groupCreate)(env, NULL, dev, 3, 10, NULL, -1.0, 1024.0, 0.51, 0.05, 100.0, 0, 1, 1, 1, 0);
  report("groupCreate");
  if (!g) return 1;
  jdoubleArray topics = arr(30, 8);
  for (int j = 0; j < 30; ++j) ((jdouble*)topics->data)[j] = 0.5 + 0.37 * (double)((j * 7) % 11);
  FN(groupSetTopics)(env, NULL, g, topics, 0);
  report("groupSetTopics");
  jdoubleArray theta = arr(9, 8);
  FN(groupTopicDistribution)(env, NULL, g, 3, 10, ip, ix, vs, 7, 100, NULL, theta);
  report("groupTopicDistribution");
  printf("theta");
  for (int j = 0; j < 9; ++j) printf("\t%.17g", ((jdouble*)theta->data)[j]);
  printf("\n");
  printf("transport\t%d\n", (int)FN(groupTransport)(env, NULL, g));
  FN(groupDestroy)(env, NULL, g);
  FN(destroy)(env, NULL, ctx);
  return 0;
}

/* GPU training mode (tests/test_gpu_jni_shim.py): the JNI calls HipOnlineLDAOptimizer makes
 * (initialize → next × steps → getLDAModel, HipOnlineLDAOptimizer.scala:105-139) and those HipLocalLDAModel
 * makes afterwards (describeTopics, logLikelihood), in the Scala code's order, over a corpus read from a
 * binary file.  Input (little-endian): int64 n_dev, n_dev device ids, rows, cols, k, steps, seed, then
 * double miniBatchFraction, then indptr[rows+1] (int64), indices[nnz] (int32), values[nnz] (double).
 * Output file: λ (V×k doubles, the k×V row-major getLDAModel reads, LAYOUT_KV), α[k], η, iteration
 * (as double), the per-step stats (steps×7 doubles), describe(10) indices (k×10 int32) and weights (k×10
 * doubles), the bound over the training rows {bound, corpus, topics, tokens}, the transport. */
static long long rd_i64(FILE* f) {
  long long v = 0;
  if (fread(&v, 8, 1, f) != 1) exit(3);
  return v;
}
static int gpu_train_main(JNIEnv* env, const char* in_path, const char* out_path) {
  FILE* f = fopen(in_path, "rb");
  if (!f) return 2;
  const long long nd = rd_i64(f);
  jintArray dev = arr((jsize)nd, 4);
  for (long long i = 0; i < nd; ++i) ((jint*)dev->data)[i] = (jint)rd_i64(f);
  const long long rows = rd_i64(f), cols = rd_i64(f), k = rd_i64(f), steps = rd_i64(f), seed = rd_i64(f);
  double frac = 0;
  if (fread(&frac, 8, 1, f) != 1) return 3;
  jlongArray ip = arr((jsize)(rows + 1), 8);
  if (fread(ip->data, 8, (size_t)(rows + 1), f) != (size_t)(rows + 1)) return 3;
  const long long nnz = ((jlong*)ip->data)[rows];
  jintArray ix = arr((jsize)nnz, 4);
  jdoubleArray vs = arr((jsize)nnz, 8);
  if (fread(ix->data, 4, (size_t)nnz, f) != (size_t)nnz || fread(vs->data, 8, (size_t)nnz, f) != (size_t)nnz) return 3;
  fclose(f);
  /* initialize(): groupCreate (α = −1 ⇒ 1/k, η = −1 ⇒ 1/k), groupSetCorpus, groupInitRandom(seed) */
  jdoubleArray alpha_in = arr(1, 8);
  ((jdouble*)alpha_in->data)[0] = -1.0;
  /* sampleWithReplacement = true: HipOnlineLDAOptimizer's (and Spark's) default; optimizeDocConcentration = true: ml LDA's */
  jlong g = FN(groupCreate)(env, NULL, dev, (jint)k, cols, alpha_in, -1.0, 1024.0, 0.51, frac, 100.0, 1, 1, seed, 1, 0);
  report("groupCreate");
  if (!g) return 1;
  FN(groupSetCorpus)(env, NULL, g, rows, cols, ip, ix, vs);
  report("groupSetCorpus");
  FN(groupInitRandom)(env, NULL, g, seed);
  report("groupInitRandom");
  /* next() × steps (with the stats array, as a caller that logs them) */
  jdoubleArray st = arr(7, 8);
  double* stats = calloc((size_t)steps * 7, 8);
  int next_ok = 1;
  for (long long s = 0; s < steps; ++s) {
    FN(groupNext)(env, NULL, g, st);
    if (g_thrown) next_ok = 0;
    report("groupNext");
    memcpy(stats + 7 * s, st->data, 7 * 8);
  }
  /* getLDAModel(): topics (k×V row-major), α, η of member 0, then the corpus released */
  jdoubleArray topics = arr((jsize)(cols * k), 8), alpha = arr((jsize)k, 8);
  FN(groupGetTopics)(env, NULL, g, topics, 1 /* LAYOUT_KV */);
  report("groupGetTopics");
  FN(groupGetAlpha)(env, NULL, g, alpha);
  report("groupGetAlpha");
  const jdouble eta = FN(ldaGetEta)(env, NULL, FN(groupMember)(env, NULL, g, 0));
  report("ldaGetEta");
  const double iteration = (double)FN(groupGetIteration)(env, NULL, g);
  report("groupGetIteration");
  FN(groupReleaseCorpus)(env, NULL, g);
  report("groupReleaseCorpus");
  /* HipLocalLDAModel: describeTopics(10), logLikelihood over the training rows (γ₀ seed 9, ids from 0) */
  jintArray didx = arr((jsize)(k * 10), 4);
  jdoubleArray dw = arr((jsize)(k * 10), 8);
  FN(groupDescribe)(env, NULL, g, 10, didx, dw);
  report("groupDescribe");
  jdoubleArray b = FN(groupBound)(env, NULL, g, rows, cols, ip, ix, vs, 9, 0, NULL);
  report("groupBound");
  const double tr = (double)FN(groupTransport)(env, NULL, g);
  FN(groupDestroy)(env, NULL, g);
  report("groupDestroy");
  FILE* o = fopen(out_path, "wb");
  if (!o) return 2;
  fwrite(topics->data, 8, (size_t)(cols * k), o);
  fwrite(alpha->data, 8, (size_t)k, o);
  fwrite(&eta, 8, 1, o);
  fwrite(&iteration, 8, 1, o);
  fwrite(stats, 8, (size_t)steps * 7, o);
  fwrite(didx->data, 4, (size_t)(k * 10), o);
  fwrite(dw->data, 8, (size_t)(k * 10), o);
  double bz[4] = {0, 0, 0, 0};
  if (b) memcpy(bz, b->data, sizeof bz);
  fwrite(bz, 8, 4, o);
  fwrite(&tr, 8, 1, o);
  fclose(o);
  free(stats);
  return next_ok ? 0 : 4;
}

int main(int argc, char** argv) {
  JNIEnv env_ = &table;
  JNIEnv* env = &env_;
  if (argc > 1 && strcmp(argv[1], "gpu") == 0) return gpu_main(env);
  if (argc > 3 && strcmp(argv[1], "gpu_train") == 0) return gpu_train_main(env, argv[2], argv[3]);
  /* 3 tokens "ab","c","" in 2 documents */
  jbyteArray utf8 = arr(3, 1);
  memcpy(utf8->data, "abc", 3);
  jlongArray tok_off = arr(4, 8), doc_off = arr(3, 8);
  jlong to[4] = {0, 2, 3, 3}, dof[3] = {0, 2, 3};
  memcpy(tok_off->data, to, sizeof to);
  memcpy(doc_off->data, dof, sizeof dof);

  FN(hashingTf)(env, NULL, 0, utf8, tok_off, doc_off, 16, 0, 0, arr(3, 8), arr(2, 4), arr(3, 8));
  report("hashingTf_short_indices");
  FN(hashingTf)(env, NULL, 0, utf8, tok_off, doc_off, 16, 0, 0, arr(2, 8), arr(3, 4), arr(3, 8));
  report("hashingTf_short_indptr");
  FN(hashingTf)(env, NULL, 0, utf8, tok_off, doc_off, 16, 0, 0, arr(3, 8), arr(3, 4), arr(3, 8));
  report("hashingTf_sized");  /* reaches the library: ctx NULL */
  FN(hashTokens)(env, NULL, 0, utf8, tok_off, 16, 0, arr(2, 4));
  report("hashTokens_short");
  {
    jbyteArray text = arr(5, 1);
    memcpy(text->data, "a b c", 5);
    jlongArray toff = arr(2, 8);
    jlong t2[2] = {0, 5};
    memcpy(toff->data, t2, sizeof t2);
    FN(tokenize)(env, NULL, 0, text, toff, arr(7, 1), arr(6, 8), arr(2, 8));
    report("tokenize_short_tokoff");
    FN(tokenize)(env, NULL, 0, text, toff, arr(6, 1), arr(7, 8), arr(2, 8));
    report("tokenize_short_utf8");
  }
  {
    jlongArray ip = arr(3, 8);
    jlong p3[3] = {0, 2, 5};
    memcpy(ip->data, p3, sizeof p3);
    FN(dcsrUpload)(env, NULL, 0, 2, 10, ip, arr(4, 4), arr(5, 8), 1);
    report("dcsrUpload_short_indices");
    FN(dcsrUpload)(env, NULL, 0, 3, 10, ip, arr(5, 4), arr(5, 8), 1);
    report("dcsrUpload_short_indptr");
  }
  FN(ldaGetTopics)(env, NULL, 0, arr(1, 8), 0);
  report("ldaGetTopics_null_handle");  /* the shape lookup fails before anything is pinned */
  FN(ldaCounters)(env, NULL, 0, arr(3, 8));
  report("ldaCounters_short");
  FN(ldaPhaseTimes)(env, NULL, 0, arr(4, 8));
  report("ldaPhaseTimes_short");
  FN(idfGet)(env, NULL, 0, 0, 10, arr(10, 8), NULL);
  report("idfGet_null_model");  /* the model's column count is looked up before anything is pinned */
  {
    jlongArray ip = arr(2, 8);
    FN(groupTopicDistribution)(env, NULL, 0, 1, 10, ip, arr(0, 4), arr(0, 8), 7, 0, NULL, arr(3, 8));
    report("groupTopicDistribution_null_group");  /* HipLDAModel.transform's call reaches the library */
  }
  return 0;
}
