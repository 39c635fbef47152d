/*
 * stcjni.c — JNI shim over libstc.so's C ABI (include/stc.h): the binding the reference's JVM side
 * (scala/…: HipOnlineLDAOptimizer at the LDAClustering.scala:40-46 optimizer switch, HipIDF at
 * LDAClustering.scala:177, the Spark-ML wrappers) calls through org.apache.spark.mllib.clustering.
 * StcNative.  One native method per stc.h entry point, same argument meaning.
 *
 * Build (needs a JDK; this container has none — `make -C jni` checks for $JAVA_HOME/include/jni.h):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../include stcjni.c \
 *       -L../spark-text-clustering_amd/stc -lstc -Wl,-rpath,'$ORIGIN' -o libstcjni.so
 *
 * Conventions:
 *   - handles (stc_ctx*, stc_dcsr*, stc_lda*) cross as jlong;
 *   - a non-zero status becomes a Java exception with stc_last_error() as the message:
 *     STC_ERR_INVALID_ARG → IllegalArgumentException, anything else → IllegalStateException;
 *   - host arrays are pinned with Get<Type>ArrayElements for the duration of the call (the library
 *     copies inputs before it returns and writes outputs before it returns); outputs are released
 *     with mode 0 (copy back), inputs with JNI_ABORT; a null Java array is passed as NULL.
 *   - every array's length is checked against the elements the C ABI will read or write (sizes from
 *     the handles: stc_lda_shape, stc_dcsr_shape) BEFORE anything is pinned: a short array throws
 *     IllegalArgumentException instead of letting the library overrun the pinned copy.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "stc.h"

#define FN(name) Java_org_apache_spark_mllib_clustering_StcNative_##name
#define CTX(h) ((stc_ctx*)(intptr_t)(h))
#define CSR(h) ((stc_dcsr*)(intptr_t)(h))
#define LDA(h) ((stc_lda*)(intptr_t)(h))
#define GRP(h) ((stc_group*)(intptr_t)(h))

static int check(JNIEnv* env, int st) {
  if (st == STC_OK) return 0;
  const char* cls = st == STC_ERR_INVALID_ARG ? "java/lang/IllegalArgumentException"
                                              : "java/lang/IllegalStateException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, stc_last_error());
  return 1;
}

/* pinned views of Java arrays (NULL-safe) */
#define PIN(T, JT, arr) ((arr) ? (T*)(*env)->Get##JT##ArrayElements(env, (arr), NULL) : (T*)NULL)
#define UNPIN(JT, arr, p, mode) \
  do {                          \
    if (arr) (*env)->Release##JT##ArrayElements(env, (arr), (void*)(p), (mode)); \
  } while (0)
#define LEN(arr) ((arr) ? (int64_t)(*env)->GetArrayLength(env, (arr)) : (int64_t)0)

static void throw_iae(JNIEnv* env, const char* msg) {
  jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (ex) (*env)->ThrowNew(env, ex, msg);
}
/* 1 (with IllegalArgumentException pending) when a non-null array holds fewer than `need` elements;
 * a null array passes (the C ABI takes NULL as "not given" and rejects it where it is required) */
static int short_array(JNIEnv* env, jarray arr, int64_t need, const char* what) {
  if (!arr) return 0;
  const int64_t n = (int64_t)(*env)->GetArrayLength(env, arr);
  if (n >= need) return 0;
  char msg[192];
  snprintf(msg, sizeof msg, "%s: the Java array has %lld elements, the call needs %lld", what, (long long)n,
           (long long)need);
  throw_iae(env, msg);
  return 1;
}
#define NEED(arr, n, what) short_array(env, (jarray)(arr), (int64_t)(n), (what))
static int lda_shape(JNIEnv* env, jlong lda, int64_t* k, int64_t* vocab) {
  int32_t kk = 0;
  int64_t vv = 0;
  if (check(env, stc_lda_shape(LDA(lda), &kk, &vv))) return 1;
  *k = kk;
  *vocab = vv;
  return 0;
}
static int csr_shape(JNIEnv* env, jlong m, int64_t* rows, int64_t* cols, int64_t* nnz) {
  return check(env, stc_dcsr_shape(CSR(m), rows, cols, nnz));
}

/* ---- library / device ------------------------------------------------------------------ */
JNIEXPORT jstring JNICALL FN(lastError)(JNIEnv* env, jclass c) {
  return (*env)->NewStringUTF(env, stc_last_error());
}

JNIEXPORT jint JNICALL FN(abiVersion)(JNIEnv* env, jclass c) { return stc_abi_version(); }

JNIEXPORT jint JNICALL FN(deviceCount)(JNIEnv* env, jclass c) {
  int n = 0;
  check(env, stc_device_count(&n));
  return n;
}

JNIEXPORT jlong JNICALL FN(init)(JNIEnv* env, jclass c, jint device) {
  stc_ctx* ctx = NULL;
  if (check(env, stc_init(device, &ctx))) return 0;
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL FN(destroy)(JNIEnv* env, jclass c, jlong ctx) { check(env, stc_destroy(CTX(ctx))); }

JNIEXPORT void JNICALL FN(synchronize)(JNIEnv* env, jclass c, jlong ctx) {
  check(env, stc_synchronize(CTX(ctx)));
}

/* ---- RCCL ---------------------------------------------------------------------------------- */
JNIEXPORT jbyteArray JNICALL FN(commUniqueId)(JNIEnv* env, jclass c) {
  uint8_t id[128];
  if (check(env, stc_comm_unique_id(id))) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, 128);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, 128, (const jbyte*)id);
  return out;
}

JNIEXPORT void JNICALL FN(commInit)(JNIEnv* env, jclass c, jlong ctx, jbyteArray id, jint n_ranks, jint rank) {
  uint8_t buf[128];
  if (LEN(id) != 128) {
    jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (ex) (*env)->ThrowNew(env, ex, "commInit: the unique id has 128 bytes");
    return;
  }
  (*env)->GetByteArrayRegion(env, id, 0, 128, (jbyte*)buf);
  check(env, stc_comm_init(CTX(ctx), buf, n_ranks, rank));
}

JNIEXPORT void JNICALL FN(commAllreduceF64)(JNIEnv* env, jclass c, jlong ctx, jdoubleArray inout) {
  jdouble* p = PIN(jdouble, Double, inout);
  int st = stc_comm_allreduce_f64(CTX(ctx), p, LEN(inout));
  UNPIN(Double, inout, p, 0);
  check(env, st);
}

/* ---- device CSR ------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL FN(dcsrUpload)(JNIEnv* env, jclass c, jlong ctx, jlong rows, jlong cols,
                                       jlongArray indptr, jintArray indices, jdoubleArray values, jint dtype) {
  stc_dcsr* out = NULL;
  if (rows < 0 || !indptr || NEED(indptr, rows + 1, "dcsrUpload indptr")) {
    if (!(*env)->ExceptionCheck(env)) throw_iae(env, "dcsrUpload: indptr[rows + 1] is required");
    return 0;
  }
  jlong last = 0;
  (*env)->GetLongArrayRegion(env, indptr, (jsize)rows, 1, &last);
  if (NEED(indices, last, "dcsrUpload indices") || NEED(values, last, "dcsrUpload values")) return 0;
  jlong* ip = PIN(jlong, Long, indptr);
  jint* ix = PIN(jint, Int, indices);
  jdouble* vs = PIN(jdouble, Double, values);
  int st = stc_dcsr_upload(CTX(ctx), rows, cols, (const int64_t*)ip, (const int32_t*)ix, vs, dtype, &out);
  UNPIN(Double, values, vs, JNI_ABORT);
  UNPIN(Int, indices, ix, JNI_ABORT);
  UNPIN(Long, indptr, ip, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

/* {rows, cols, nnz} */
JNIEXPORT jlongArray JNICALL FN(dcsrShape)(JNIEnv* env, jclass c, jlong m) {
  int64_t s[3] = {0, 0, 0};
  if (check(env, stc_dcsr_shape(CSR(m), &s[0], &s[1], &s[2]))) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 3);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 3, (const jlong*)s);
  return out;
}

JNIEXPORT void JNICALL FN(dcsrDownload)(JNIEnv* env, jclass c, jlong ctx, jlong m, jlongArray indptr,
                                        jintArray indices, jdoubleArray values) {
  int64_t rows = 0, cols = 0, nnz = 0;
  if (csr_shape(env, m, &rows, &cols, &nnz) || NEED(indptr, rows + 1, "dcsrDownload indptr") ||
      NEED(indices, nnz, "dcsrDownload indices") || NEED(values, nnz, "dcsrDownload values"))
    return;
  jlong* ip = PIN(jlong, Long, indptr);
  jint* ix = PIN(jint, Int, indices);
  jdouble* vs = PIN(jdouble, Double, values);
  int st = stc_dcsr_download(CTX(ctx), CSR(m), (int64_t*)ip, (int32_t*)ix, vs);
  UNPIN(Double, values, vs, 0);
  UNPIN(Int, indices, ix, 0);
  UNPIN(Long, indptr, ip, 0);
  check(env, st);
}

JNIEXPORT void JNICALL FN(dcsrFree)(JNIEnv* env, jclass c, jlong m) { check(env, stc_dcsr_free(CSR(m))); }

/* ---- HashingTF -------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL FN(hashingTfDev)(JNIEnv* env, jclass c, jlong ctx, jbyteArray utf8, jlongArray tok_off,
                                         jlongArray doc_off, jint num_features, jboolean binary, jint variant,
                                         jint dtype) {
  stc_dcsr* out = NULL;
  jbyte* u = PIN(jbyte, Byte, utf8);
  jlong* to = PIN(jlong, Long, tok_off);
  jlong* dof = PIN(jlong, Long, doc_off);
  int st = stc_hashing_tf_dev(CTX(ctx), (const uint8_t*)u, LEN(utf8), (const int64_t*)to, LEN(tok_off) - 1,
                              (const int64_t*)dof, LEN(doc_off) - 1, num_features, binary, variant, dtype, &out);
  UNPIN(Long, doc_off, dof, JNI_ABORT);
  UNPIN(Long, tok_off, to, JNI_ABORT);
  UNPIN(Byte, utf8, u, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

JNIEXPORT void JNICALL FN(hashingTf)(JNIEnv* env, jclass c, jlong ctx, jbyteArray utf8, jlongArray tok_off,
                                     jlongArray doc_off, jint num_features, jboolean binary, jint variant,
                                     jlongArray indptr_out, jintArray indices_out, jdoubleArray values_out) {
  const int64_t n_tok = LEN(tok_off) - 1, n_docs = LEN(doc_off) - 1;
  if (NEED(indptr_out, n_docs + 1, "hashingTf indptrOut") || NEED(indices_out, n_tok, "hashingTf indicesOut") ||
      NEED(values_out, n_tok, "hashingTf valuesOut"))
    return;
  jbyte* u = PIN(jbyte, Byte, utf8);
  jlong* to = PIN(jlong, Long, tok_off);
  jlong* dof = PIN(jlong, Long, doc_off);
  jlong* ip = PIN(jlong, Long, indptr_out);
  jint* ix = PIN(jint, Int, indices_out);
  jdouble* vs = PIN(jdouble, Double, values_out);
  int st = stc_hashing_tf(CTX(ctx), (const uint8_t*)u, LEN(utf8), (const int64_t*)to, LEN(tok_off) - 1,
                          (const int64_t*)dof, LEN(doc_off) - 1, num_features, binary, variant, (int64_t*)ip,
                          (int32_t*)ix, vs);
  UNPIN(Double, values_out, vs, 0);
  UNPIN(Int, indices_out, ix, 0);
  UNPIN(Long, indptr_out, ip, 0);
  UNPIN(Long, doc_off, dof, JNI_ABORT);
  UNPIN(Long, tok_off, to, JNI_ABORT);
  UNPIN(Byte, utf8, u, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(hashTokens)(JNIEnv* env, jclass c, jlong ctx, jbyteArray utf8, jlongArray tok_off,
                                      jint num_features, jint variant, jintArray idx_out) {
  if (NEED(idx_out, LEN(tok_off) - 1, "hashTokens idxOut")) return;
  jbyte* u = PIN(jbyte, Byte, utf8);
  jlong* to = PIN(jlong, Long, tok_off);
  jint* ix = PIN(jint, Int, idx_out);
  int st = stc_hash_tokens(CTX(ctx), (const uint8_t*)u, LEN(utf8), (const int64_t*)to, LEN(tok_off) - 1,
                           num_features, variant, (int32_t*)ix);
  UNPIN(Int, idx_out, ix, 0);
  UNPIN(Long, tok_off, to, JNI_ABORT);
  UNPIN(Byte, utf8, u, JNI_ABORT);
  check(env, st);
}

JNIEXPORT jlong JNICALL FN(tokensUpload)(JNIEnv* env, jclass c, jlong ctx, jbyteArray utf8, jlongArray tok_off,
                                         jlongArray doc_off) {
  stc_dtok* out = NULL;
  jbyte* u = PIN(jbyte, Byte, utf8);
  jlong* to = PIN(jlong, Long, tok_off);
  jlong* dof = PIN(jlong, Long, doc_off);
  int st = stc_tokens_upload(CTX(ctx), (const uint8_t*)u, LEN(utf8), (const int64_t*)to, LEN(tok_off) - 1,
                             (const int64_t*)dof, LEN(doc_off) - 1, &out);
  UNPIN(Long, doc_off, dof, JNI_ABORT);
  UNPIN(Long, tok_off, to, JNI_ABORT);
  UNPIN(Byte, utf8, u, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

JNIEXPORT void JNICALL FN(tokensFree)(JNIEnv* env, jclass c, jlong tokens) {
  check(env, stc_tokens_free((stc_dtok*)(intptr_t)tokens));
}

JNIEXPORT jlong JNICALL FN(hashingTfTokens)(JNIEnv* env, jclass c, jlong ctx, jlong tokens, jint num_features,
                                            jboolean binary, jint variant, jint dtype) {
  stc_dcsr* out = NULL;
  if (check(env, stc_hashing_tf_tokens(CTX(ctx), (const stc_dtok*)(intptr_t)tokens, num_features, binary,
                                       variant, dtype, &out)))
    return 0;
  return (jlong)(intptr_t)out;
}

/* ---- Tokenizer -------------------------------------------------------------------------- */
/* outputs sized by the caller: utf8Out ≥ text.length * 3 / 2, tokOffOut ≥ text.length + nDocs + 1,
 * docOffOut = nDocs + 1; returns {nOutBytes, nTok} */
JNIEXPORT jlongArray JNICALL FN(tokenize)(JNIEnv* env, jclass c, jlong ctx, jbyteArray text, jlongArray text_off,
                                          jbyteArray utf8_out, jlongArray tok_off_out, jlongArray doc_off_out) {
  int64_t nb = 0, nt = 0;
  const int64_t n_bytes = LEN(text), n_docs = LEN(text_off) - 1;
  if (NEED(utf8_out, n_bytes + n_bytes / 2, "tokenize utf8Out") || NEED(tok_off_out, n_bytes + n_docs + 1, "tokenize tokOffOut") ||
      NEED(doc_off_out, n_docs + 1, "tokenize docOffOut"))
    return NULL;
  jbyte* t = PIN(jbyte, Byte, text);
  jlong* off = PIN(jlong, Long, text_off);
  jbyte* u = PIN(jbyte, Byte, utf8_out);
  jlong* to = PIN(jlong, Long, tok_off_out);
  jlong* dof = PIN(jlong, Long, doc_off_out);
  int st = stc_tokenize(CTX(ctx), (const uint8_t*)t, LEN(text), (const int64_t*)off, LEN(text_off) - 1,
                        (uint8_t*)u, LEN(utf8_out), &nb, (int64_t*)to, &nt, (int64_t*)dof);
  UNPIN(Long, doc_off_out, dof, 0);
  UNPIN(Long, tok_off_out, to, 0);
  UNPIN(Byte, utf8_out, u, 0);
  UNPIN(Long, text_off, off, JNI_ABORT);
  UNPIN(Byte, text, t, JNI_ABORT);
  if (check(env, st)) return NULL;
  int64_t r[2] = {nb, nt};
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, (const jlong*)r);
  return out;
}

JNIEXPORT jlong JNICALL FN(tokenizeHashingTfDev)(JNIEnv* env, jclass c, jlong ctx, jbyteArray text,
                                                 jlongArray text_off, jint num_features, jboolean binary,
                                                 jint variant, jint dtype) {
  stc_dcsr* out = NULL;
  jbyte* t = PIN(jbyte, Byte, text);
  jlong* off = PIN(jlong, Long, text_off);
  int st = stc_tokenize_hashing_tf_dev(CTX(ctx), (const uint8_t*)t, LEN(text), (const int64_t*)off,
                                       LEN(text_off) - 1, num_features, binary, variant, dtype, &out);
  UNPIN(Long, text_off, off, JNI_ABORT);
  UNPIN(Byte, text, t, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

/* ---- IDF -------------------------------------------------------------------------------- */
/* idfOut[numCols], dfOut[numCols] (may be null); returns m */
JNIEXPORT jlong JNICALL FN(idfFit)(JNIEnv* env, jclass c, jlong ctx, jlong dcsr, jlong min_doc_freq,
                                   jdoubleArray idf_out, jlongArray df_out) {
  int64_t m = 0, rows = 0, cols = 0, nnz = 0;
  if (csr_shape(env, dcsr, &rows, &cols, &nnz) || NEED(idf_out, cols, "idfFit idfOut") ||
      NEED(df_out, cols, "idfFit dfOut"))
    return 0;
  jdouble* o = PIN(jdouble, Double, idf_out);
  jlong* df = PIN(jlong, Long, df_out);
  int st = stc_idf_fit(CTX(ctx), CSR(dcsr), min_doc_freq, o, (int64_t*)df, &m);
  UNPIN(Long, df_out, df, 0);
  UNPIN(Double, idf_out, o, 0);
  if (check(env, st)) return 0;
  return m;
}

JNIEXPORT void JNICALL FN(idfTransform)(JNIEnv* env, jclass c, jlong ctx, jlong dcsr, jdoubleArray idf,
                                        jdouble zero_floor) {
  int64_t rows = 0, cols = 0, nnz = 0;
  if (csr_shape(env, dcsr, &rows, &cols, &nnz) || NEED(idf, cols, "idfTransform idf")) return;
  jdouble* p = PIN(jdouble, Double, idf);
  int st = stc_idf_transform(CTX(ctx), CSR(dcsr), p, zero_floor);
  UNPIN(Double, idf, p, JNI_ABORT);
  check(env, st);
}

/* the IDF model kept on the device (GPU-resident pipeline); idfGet copies it out: returns m */
JNIEXPORT jlong JNICALL FN(idfFitDev)(JNIEnv* env, jclass c, jlong ctx, jlong dcsr, jlong min_doc_freq) {
  stc_didf* md = NULL;
  if (check(env, stc_idf_fit_dev(CTX(ctx), CSR(dcsr), min_doc_freq, &md))) return 0;
  return (jlong)(intptr_t)md;
}

JNIEXPORT jlong JNICALL FN(idfGet)(JNIEnv* env, jclass c, jlong ctx, jlong model, jlong cols, jdoubleArray idf_out,
                                   jlongArray df_out) {
  int64_t m = 0, mcols = 0;
  /* stc_idf_get writes the MODEL's column count into each output: size the checks from the model, and
   * refuse a caller whose idea of numFeatures differs (a smaller `cols` overran the array) */
  if (check(env, stc_didf_shape((const stc_didf*)(intptr_t)model, &mcols, NULL))) return 0;
  if (cols != mcols) {
    char msg[160];
    snprintf(msg, sizeof msg, "idfGet: cols = %lld, the model has %lld columns", (long long)cols, (long long)mcols);
    throw_iae(env, msg);
    return 0;
  }
  if ((idf_out && NEED(idf_out, mcols, "idfGet idfOut")) || (df_out && NEED(df_out, mcols, "idfGet dfOut"))) return 0;
  jdouble* o = idf_out ? PIN(jdouble, Double, idf_out) : NULL;
  jlong* df = df_out ? PIN(jlong, Long, df_out) : NULL;
  int st = stc_idf_get(CTX(ctx), (const stc_didf*)(intptr_t)model, o, (int64_t*)df, &m);
  if (df) UNPIN(Long, df_out, df, 0);
  if (o) UNPIN(Double, idf_out, o, 0);
  if (check(env, st)) return 0;
  return m;
}

JNIEXPORT void JNICALL FN(idfTransformDev)(JNIEnv* env, jclass c, jlong ctx, jlong dcsr, jlong model,
                                           jdouble zero_floor) {
  check(env, stc_idf_transform_dev(CTX(ctx), CSR(dcsr), (const stc_didf*)(intptr_t)model, zero_floor));
}

/* {numFeatures, m} of a device IDF model */
JNIEXPORT jlongArray JNICALL FN(didfShape)(JNIEnv* env, jclass c, jlong model) {
  int64_t s[2] = {0, 0};
  if (check(env, stc_didf_shape((const stc_didf*)(intptr_t)model, &s[0], &s[1]))) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, (const jlong*)s);
  return out;
}

JNIEXPORT void JNICALL FN(didfFree)(JNIEnv* env, jclass c, jlong model) {
  check(env, stc_didf_free((stc_didf*)(intptr_t)model));
}

/* ---- online LDA ------------------------------------------------------------------------- */
/* stc_lda_config_default + the given fields (alpha: length 1 or k, or null ⇒ −1 ⇒ 1/k) */
JNIEXPORT jlong JNICALL FN(ldaCreate)(JNIEnv* env, jclass c, jlong ctx, jint k, jlong vocab, jdoubleArray alpha,
                                      jdouble eta, jdouble tau0, jdouble kappa, jdouble frac, jdouble gamma_shape,
                                      jboolean optimize_alpha, jboolean with_replacement, jlong seed, jint dtype,
                                      jint max_inner_iter) {
  stc_lda_config cfg;
  stc_lda_config_default(&cfg);
  jdouble* a = PIN(jdouble, Double, alpha);
  cfg.k = k;
  cfg.vocab_size = vocab;
  cfg.doc_concentration = a;
  cfg.doc_concentration_len = (int32_t)LEN(alpha);
  cfg.topic_concentration = eta;
  cfg.tau0 = tau0;
  cfg.kappa = kappa;
  cfg.mini_batch_fraction = frac;
  cfg.gamma_shape = gamma_shape;
  cfg.optimize_doc_concentration = optimize_alpha ? 1 : 0;
  cfg.sample_with_replacement = with_replacement ? 1 : 0;
  cfg.seed = (uint64_t)seed;
  cfg.dtype = dtype;
  cfg.max_inner_iter = max_inner_iter;
  stc_lda* out = NULL;
  int st = stc_lda_create(CTX(ctx), &cfg, &out); /* resolves and copies α */
  UNPIN(Double, alpha, a, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

JNIEXPORT void JNICALL FN(ldaDestroy)(JNIEnv* env, jclass c, jlong lda) { check(env, stc_lda_destroy(LDA(lda))); }

JNIEXPORT void JNICALL FN(ldaSetCorpus)(JNIEnv* env, jclass c, jlong lda, jlong dcsr, jlong total) {
  check(env, stc_lda_set_corpus(LDA(lda), CSR(dcsr), total));
}

JNIEXPORT void JNICALL FN(ldaInitRandom)(JNIEnv* env, jclass c, jlong lda, jlong seed) {
  check(env, stc_lda_init_random(LDA(lda), (uint64_t)seed));
}

JNIEXPORT void JNICALL FN(ldaSetTopics)(JNIEnv* env, jclass c, jlong lda, jdoubleArray topics, jint layout) {
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V) || NEED(topics, k * V, "ldaSetTopics topics")) return;
  jdouble* p = PIN(jdouble, Double, topics);
  int st = stc_lda_set_topics(LDA(lda), p, layout);
  UNPIN(Double, topics, p, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(ldaGetTopics)(JNIEnv* env, jclass c, jlong lda, jdoubleArray out, jint layout) {
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V) || NEED(out, k * V, "ldaGetTopics out")) return;
  jdouble* p = PIN(jdouble, Double, out);
  int st = stc_lda_get_topics(LDA(lda), p, layout);
  UNPIN(Double, out, p, 0);
  check(env, st);
}

JNIEXPORT void JNICALL FN(ldaSetAlpha)(JNIEnv* env, jclass c, jlong lda, jdoubleArray alpha) {
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V) || NEED(alpha, k, "ldaSetAlpha alpha")) return;
  jdouble* p = PIN(jdouble, Double, alpha);
  int st = stc_lda_set_alpha(LDA(lda), p);
  UNPIN(Double, alpha, p, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(ldaGetAlpha)(JNIEnv* env, jclass c, jlong lda, jdoubleArray out) {
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V) || NEED(out, k, "ldaGetAlpha out")) return;
  jdouble* p = PIN(jdouble, Double, out);
  int st = stc_lda_get_alpha(LDA(lda), p);
  UNPIN(Double, out, p, 0);
  check(env, st);
}

JNIEXPORT jdouble JNICALL FN(ldaGetEta)(JNIEnv* env, jclass c, jlong lda) {
  double eta = 0.0;
  check(env, stc_lda_get_eta(LDA(lda), &eta));
  return eta;
}

JNIEXPORT jlong JNICALL FN(ldaGetIteration)(JNIEnv* env, jclass c, jlong lda) {
  int64_t it = 0;
  check(env, stc_lda_get_iteration(LDA(lda), &it));
  return it;
}

/* {k, vocabSize} */
JNIEXPORT jlongArray JNICALL FN(ldaShape)(JNIEnv* env, jclass c, jlong lda) {
  int64_t s[2] = {0, 0};
  if (lda_shape(env, lda, &s[0], &s[1])) return NULL;
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, (const jlong*)s);
  return out;
}

/* step statistics as doubles: {batchDocs, nonemptyDocs, batchEntries, innerIters, innerItersMax,
 * capHits, rho} */
static void stats_out(JNIEnv* env, jdoubleArray out, const stc_step_stats* s) {
  if (!out || LEN(out) < 7) return;
  const jdouble v[7] = {(double)s->batch_docs, (double)s->nonempty_docs, (double)s->batch_entries,
                        (double)s->inner_iters, (double)s->inner_iters_max, (double)s->cap_hits, s->rho};
  (*env)->SetDoubleArrayRegion(env, out, 0, 7, v);
}

JNIEXPORT void JNICALL FN(ldaStep)(JNIEnv* env, jclass c, jlong lda, jlongArray ids, jdoubleArray gamma0,
                                   jdoubleArray stats) {
  stc_step_stats s;
  memset(&s, 0, sizeof s);
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V) || NEED(gamma0, LEN(ids) * k, "ldaStep gamma0")) return;
  jlong* p = PIN(jlong, Long, ids);
  jdouble* g = PIN(jdouble, Double, gamma0);
  int st = stc_lda_step(LDA(lda), (const int64_t*)p, LEN(ids), g, stats ? &s : NULL);
  UNPIN(Double, gamma0, g, JNI_ABORT);
  UNPIN(Long, ids, p, JNI_ABORT);
  if (!check(env, st)) stats_out(env, stats, &s);
}

JNIEXPORT void JNICALL FN(ldaNext)(JNIEnv* env, jclass c, jlong lda, jdoubleArray stats) {
  stc_step_stats s;
  memset(&s, 0, sizeof s);
  if (!check(env, stc_lda_next(LDA(lda), stats ? &s : NULL))) stats_out(env, stats, &s);
}

JNIEXPORT void JNICALL FN(ldaEstep)(JNIEnv* env, jclass c, jlong lda, jlongArray ids, jdoubleArray gamma0,
                                    jdoubleArray gamma_out, jdoubleArray stat_out, jintArray iters_out) {
  int64_t k = 0, V = 0;
  const int64_t n = LEN(ids);
  if (lda_shape(env, lda, &k, &V) || NEED(gamma0, n * k, "ldaEstep gamma0") ||
      NEED(gamma_out, n * k, "ldaEstep gammaOut") || NEED(stat_out, V * k, "ldaEstep statOut") ||
      NEED(iters_out, n, "ldaEstep itersOut"))
    return;
  jlong* p = PIN(jlong, Long, ids);
  jdouble* g0 = PIN(jdouble, Double, gamma0);
  jdouble* g = PIN(jdouble, Double, gamma_out);
  jdouble* sv = PIN(jdouble, Double, stat_out);
  jint* it = PIN(jint, Int, iters_out);
  int st = stc_lda_estep(LDA(lda), (const int64_t*)p, LEN(ids), g0, g, sv, (int32_t*)it);
  UNPIN(Int, iters_out, it, 0);
  UNPIN(Double, stat_out, sv, 0);
  UNPIN(Double, gamma_out, g, 0);
  UNPIN(Double, gamma0, g0, JNI_ABORT);
  UNPIN(Long, ids, p, JNI_ABORT);
  check(env, st);
}

/* {bound, corpusPart, topicsPart, tokenCount} */
JNIEXPORT jdoubleArray JNICALL FN(ldaBound)(JNIEnv* env, jclass c, jlong lda, jlong dcsr, jlong gamma_seed,
                                            jlong doc_id_base, jdoubleArray gamma0) {
  double r[4] = {0, 0, 0, 0};
  int64_t k = 0, V = 0, rows = 0, cols = 0, nnz = 0;
  if (lda_shape(env, lda, &k, &V) || csr_shape(env, dcsr, &rows, &cols, &nnz) ||
      NEED(gamma0, rows * k, "ldaBound gamma0"))
    return NULL;
  jdouble* g = PIN(jdouble, Double, gamma0);
  int st = stc_lda_bound(LDA(lda), CSR(dcsr), (uint64_t)gamma_seed, doc_id_base, g, &r[0], &r[1], &r[2], &r[3]);
  UNPIN(Double, gamma0, g, JNI_ABORT);
  if (check(env, st)) return NULL;
  jdoubleArray out = (*env)->NewDoubleArray(env, 4);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, 4, r);
  return out;
}

JNIEXPORT void JNICALL FN(ldaTopicDistribution)(JNIEnv* env, jclass c, jlong lda, jlong dcsr, jlong gamma_seed,
                                                jlong doc_id_base, jdoubleArray gamma0, jdoubleArray out) {
  int64_t k = 0, V = 0, rows = 0, cols = 0, nnz = 0;
  if (lda_shape(env, lda, &k, &V) || csr_shape(env, dcsr, &rows, &cols, &nnz) ||
      NEED(gamma0, rows * k, "ldaTopicDistribution gamma0") || NEED(out, rows * k, "ldaTopicDistribution out"))
    return;
  jdouble* g = PIN(jdouble, Double, gamma0);
  jdouble* o = PIN(jdouble, Double, out);
  int st = stc_lda_topic_distribution(LDA(lda), CSR(dcsr), (uint64_t)gamma_seed, doc_id_base, g, o);
  UNPIN(Double, out, o, 0);
  UNPIN(Double, gamma0, g, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(ldaDescribe)(JNIEnv* env, jclass c, jlong lda, jint max_terms, jintArray idx_out,
                                       jdoubleArray weight_out) {
  int64_t k = 0, V = 0;
  if (lda_shape(env, lda, &k, &V)) return;
  const int64_t N = max_terms < V ? (max_terms > 0 ? max_terms : 0) : V;
  if (NEED(idx_out, k * N, "ldaDescribe idxOut") || NEED(weight_out, k * N, "ldaDescribe weightOut")) return;
  jint* ix = PIN(jint, Int, idx_out);
  jdouble* w = PIN(jdouble, Double, weight_out);
  int st = stc_lda_describe(LDA(lda), max_terms, (int32_t*)ix, w);
  UNPIN(Double, weight_out, w, 0);
  UNPIN(Int, idx_out, ix, 0);
  check(env, st);
}

JNIEXPORT void JNICALL FN(ldaEnableTiming)(JNIEnv* env, jclass c, jlong lda, jboolean on) {
  check(env, stc_lda_enable_timing(LDA(lda), on ? 1 : 0));
}

JNIEXPORT void JNICALL FN(ldaCounters)(JNIEnv* env, jclass c, jlong lda, jlongArray out) {
  if (NEED(out, 4, "ldaCounters out")) return;
  jlong* p = PIN(jlong, Long, out);
  int st = stc_lda_counters(LDA(lda), (int64_t*)p);
  UNPIN(Long, out, p, 0);
  check(env, st);
}

/* out[12]: E-step launches per kernel family (stc.h enum stc_kernel_count) */
JNIEXPORT void JNICALL FN(ldaKernelCounts)(JNIEnv* env, jclass c, jlong lda, jlongArray out) {
  if (NEED(out, STC_KC_N, "ldaKernelCounts out")) return;
  jlong* p = PIN(jlong, Long, out);
  int st = stc_lda_kernel_counts(LDA(lda), (int64_t*)p);
  UNPIN(Long, out, p, 0);
  check(env, st);
}

/* msOut[5]; returns the number of timed steps */
JNIEXPORT jlong JNICALL FN(ldaPhaseTimes)(JNIEnv* env, jclass c, jlong lda, jdoubleArray ms_out) {
  int64_t steps = 0;
  if (NEED(ms_out, 5, "ldaPhaseTimes msOut")) return 0;
  jdouble* p = PIN(jdouble, Double, ms_out);
  int st = stc_lda_phase_times(LDA(lda), p, &steps);
  UNPIN(Double, ms_out, p, 0);
  check(env, st);
  return steps;
}

/* ---- one process, N devices (stc_group) ---------------------------------------------------------- */
/* the same parameters as ldaCreate, plus the device ids */
JNIEXPORT jlong JNICALL FN(groupCreate)(JNIEnv* env, jclass c, jintArray devices, jint k, jlong vocab,
                                        jdoubleArray alpha, jdouble eta, jdouble tau0, jdouble kappa, jdouble frac,
                                        jdouble gamma_shape, jboolean optimize_alpha, jboolean with_replacement,
                                        jlong seed, jint dtype, jint max_inner_iter) {
  if (!devices || LEN(devices) < 1) {
    throw_iae(env, "groupCreate: at least one device id");
    return 0;
  }
  stc_lda_config cfg;
  stc_lda_config_default(&cfg);
  jdouble* a = PIN(jdouble, Double, alpha);
  jint* dv = PIN(jint, Int, devices);
  cfg.k = k;
  cfg.vocab_size = vocab;
  cfg.doc_concentration = a;
  cfg.doc_concentration_len = (int32_t)LEN(alpha);
  cfg.topic_concentration = eta;
  cfg.tau0 = tau0;
  cfg.kappa = kappa;
  cfg.mini_batch_fraction = frac;
  cfg.gamma_shape = gamma_shape;
  cfg.optimize_doc_concentration = optimize_alpha ? 1 : 0;
  cfg.sample_with_replacement = with_replacement ? 1 : 0;
  cfg.seed = (uint64_t)seed;
  cfg.dtype = dtype;
  cfg.max_inner_iter = max_inner_iter;
  stc_group* out = NULL;
  int st = stc_group_create((const int*)dv, (int)LEN(devices), &cfg, &out);
  UNPIN(Int, devices, dv, JNI_ABORT);
  UNPIN(Double, alpha, a, JNI_ABORT);
  if (check(env, st)) return 0;
  return (jlong)(intptr_t)out;
}

JNIEXPORT void JNICALL FN(groupDestroy)(JNIEnv* env, jclass c, jlong g) { check(env, stc_group_destroy(GRP(g))); }

JNIEXPORT jint JNICALL FN(groupSize)(JNIEnv* env, jclass c, jlong g) {
  int n = 0;
  check(env, stc_group_size(GRP(g), &n));
  return n;
}

/* STC_TRANSPORT_NONE / _IN_PROCESS / _RCCL */
JNIEXPORT jint JNICALL FN(groupTransport)(JNIEnv* env, jclass c, jlong g) {
  int t = 0;
  check(env, stc_group_transport(GRP(g), &t));
  return t;
}

JNIEXPORT jlong JNICALL FN(groupMember)(JNIEnv* env, jclass c, jlong g, jint i) {
  stc_lda* l = NULL;
  if (check(env, stc_group_member(GRP(g), i, &l))) return 0;
  return (jlong)(intptr_t)l;
}

/* the host CSR of a group call: indptr[rows + 1], indices / values[indptr[rows]] */
static int csr_args(JNIEnv* env, jlong rows, jlongArray indptr, jintArray indices, jdoubleArray values,
                    const char* what) {
  if (rows < 0 || !indptr || NEED(indptr, rows + 1, what)) {
    if (!(*env)->ExceptionCheck(env)) throw_iae(env, "indptr[rows + 1] is required");
    return 1;
  }
  jlong last = 0;
  (*env)->GetLongArrayRegion(env, indptr, (jsize)rows, 1, &last);
  return NEED(indices, last, what) || NEED(values, last, what);
}

JNIEXPORT void JNICALL FN(groupSetCorpus)(JNIEnv* env, jclass c, jlong g, jlong rows, jlong cols, jlongArray indptr,
                                          jintArray indices, jdoubleArray values) {
  if (csr_args(env, rows, indptr, indices, values, "groupSetCorpus")) return;
  jlong* ip = PIN(jlong, Long, indptr);
  jint* ix = PIN(jint, Int, indices);
  jdouble* vs = PIN(jdouble, Double, values);
  int st = stc_group_set_corpus(GRP(g), rows, cols, (const int64_t*)ip, (const int32_t*)ix, vs);
  UNPIN(Double, values, vs, JNI_ABORT);
  UNPIN(Int, indices, ix, JNI_ABORT);
  UNPIN(Long, indptr, ip, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(groupSynchronize)(JNIEnv* env, jclass c, jlong g) { check(env, stc_group_synchronize(GRP(g))); }

JNIEXPORT void JNICALL FN(groupReleaseCorpus)(JNIEnv* env, jclass c, jlong g) {
  check(env, stc_group_release_corpus(GRP(g)));
}

JNIEXPORT void JNICALL FN(groupInitRandom)(JNIEnv* env, jclass c, jlong g, jlong seed) {
  check(env, stc_group_init_random(GRP(g), (uint64_t)seed));
}

static int group_shape(JNIEnv* env, jlong g, int64_t* k, int64_t* vocab) {
  stc_lda* l = NULL;
  if (check(env, stc_group_member(GRP(g), 0, &l))) return 1;
  return lda_shape(env, (jlong)(intptr_t)l, k, vocab);
}

JNIEXPORT void JNICALL FN(groupSetTopics)(JNIEnv* env, jclass c, jlong g, jdoubleArray topics, jint layout) {
  int64_t k = 0, V = 0;
  if (group_shape(env, g, &k, &V) || NEED(topics, k * V, "groupSetTopics topics")) return;
  jdouble* p = PIN(jdouble, Double, topics);
  int st = stc_group_set_topics(GRP(g), p, layout);
  UNPIN(Double, topics, p, JNI_ABORT);
  check(env, st);
}

JNIEXPORT void JNICALL FN(groupGetTopics)(JNIEnv* env, jclass c, jlong g, jdoubleArray out, jint layout) {
  int64_t k = 0, V = 0;
  if (group_shape(env, g, &k, &V) || NEED(out, k * V, "groupGetTopics out")) return;
  jdouble* p = PIN(jdouble, Double, out);
  int st = stc_group_get_topics(GRP(g), p, layout);
  UNPIN(Double, out, p, 0);
  check(env, st);
}

JNIEXPORT void JNICALL FN(groupGetAlpha)(JNIEnv* env, jclass c, jlong g, jdoubleArray out) {
  int64_t k = 0, V = 0;
  if (group_shape(env, g, &k, &V) || NEED(out, k, "groupGetAlpha out")) return;
  jdouble* p = PIN(jdouble, Double, out);
  int st = stc_group_get_alpha(GRP(g), p);
  UNPIN(Double, out, p, 0);
  check(env, st);
}

JNIEXPORT jlong JNICALL FN(groupGetIteration)(JNIEnv* env, jclass c, jlong g) {
  int64_t it = 0;
  check(env, stc_group_get_iteration(GRP(g), &it));
  return it;
}

JNIEXPORT void JNICALL FN(groupNext)(JNIEnv* env, jclass c, jlong g, jdoubleArray stats) {
  stc_step_stats s;
  memset(&s, 0, sizeof s);
  if (!check(env, stc_group_next(GRP(g), stats ? &s : NULL))) stats_out(env, stats, &s);
}

JNIEXPORT void JNICALL FN(groupStep)(JNIEnv* env, jclass c, jlong g, jlongArray ids, jdoubleArray gamma0,
                                     jdoubleArray stats) {
  stc_step_stats s;
  memset(&s, 0, sizeof s);
  int64_t k = 0, V = 0;
  if (group_shape(env, g, &k, &V) || NEED(gamma0, LEN(ids) * k, "groupStep gamma0")) return;
  jlong* p = PIN(jlong, Long, ids);
  jdouble* g0 = PIN(jdouble, Double, gamma0);
  int st = stc_group_step(GRP(g), (const int64_t*)p, LEN(ids), g0, stats ? &s : NULL);
  UNPIN(Double, gamma0, g0, JNI_ABORT);
  UNPIN(Long, ids, p, JNI_ABORT);
  if (!check(env, st)) stats_out(env, stats, &s);
}

JNIEXPORT void JNICALL FN(groupDescribe)(JNIEnv* env, jclass c, jlong g, jint max_terms, jintArray idx_out,
                                         jdoubleArray weight_out) {
  int64_t k = 0, V = 0;
  if (group_shape(env, g, &k, &V)) return;
  const int64_t N = max_terms < V ? (max_terms > 0 ? max_terms : 0) : V;
  if (NEED(idx_out, k * N, "groupDescribe idxOut") || NEED(weight_out, k * N, "groupDescribe weightOut")) return;
  jint* ix = PIN(jint, Int, idx_out);
  jdouble* w = PIN(jdouble, Double, weight_out);
  int st = stc_group_describe(GRP(g), max_terms, (int32_t*)ix, w);
  UNPIN(Double, weight_out, w, 0);
  UNPIN(Int, idx_out, ix, 0);
  check(env, st);
}

/* {bound, corpusPart, topicsPart, tokenCount} */
JNIEXPORT jdoubleArray JNICALL FN(groupBound)(JNIEnv* env, jclass c, jlong g, jlong rows, jlong cols,
                                              jlongArray indptr, jintArray indices, jdoubleArray values,
                                              jlong gamma_seed, jlong doc_id_base, jdoubleArray gamma0) {
  int64_t k = 0, V = 0;
  if (csr_args(env, rows, indptr, indices, values, "groupBound") || group_shape(env, g, &k, &V) ||
      NEED(gamma0, rows * k, "groupBound gamma0"))
    return NULL;
  double r[4] = {0, 0, 0, 0};
  jlong* ip = PIN(jlong, Long, indptr);
  jint* ix = PIN(jint, Int, indices);
  jdouble* vs = PIN(jdouble, Double, values);
  jdouble* g0 = PIN(jdouble, Double, gamma0);
  int st = stc_group_bound(GRP(g), rows, cols, (const int64_t*)ip, (const int32_t*)ix, vs, (uint64_t)gamma_seed,
                           doc_id_base, g0, &r[0], &r[1], &r[2], &r[3]);
  UNPIN(Double, gamma0, g0, JNI_ABORT);
  UNPIN(Double, values, vs, JNI_ABORT);
  UNPIN(Int, indices, ix, JNI_ABORT);
  UNPIN(Long, indptr, ip, JNI_ABORT);
  if (check(env, st)) return NULL;
  jdoubleArray out = (*env)->NewDoubleArray(env, 4);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, 4, r);
  return out;
}

JNIEXPORT void JNICALL FN(groupTopicDistribution)(JNIEnv* env, jclass c, jlong g, jlong rows, jlong cols,
                                                  jlongArray indptr, jintArray indices, jdoubleArray values,
                                                  jlong gamma_seed, jlong doc_id_base, jdoubleArray gamma0,
                                                  jdoubleArray out) {
  int64_t k = 0, V = 0;
  if (csr_args(env, rows, indptr, indices, values, "groupTopicDistribution") || group_shape(env, g, &k, &V) ||
      NEED(gamma0, rows * k, "groupTopicDistribution gamma0") || NEED(out, rows * k, "groupTopicDistribution out"))
    return;
  jlong* ip = PIN(jlong, Long, indptr);
  jint* ix = PIN(jint, Int, indices);
  jdouble* vs = PIN(jdouble, Double, values);
  jdouble* g0 = PIN(jdouble, Double, gamma0);
  jdouble* o = PIN(jdouble, Double, out);
  int st = stc_group_topic_distribution(GRP(g), rows, cols, (const int64_t*)ip, (const int32_t*)ix, vs,
                                        (uint64_t)gamma_seed, doc_id_base, g0, o);
  UNPIN(Double, out, o, 0);
  UNPIN(Double, gamma0, g0, JNI_ABORT);
  UNPIN(Double, values, vs, JNI_ABORT);
  UNPIN(Int, indices, ix, JNI_ABORT);
  UNPIN(Long, indptr, ip, JNI_ABORT);
  check(env, st);
}
