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

int main(void) {
  JNIEnv env_ = &table;
  JNIEnv* env = &env_;
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
  return 0;
}
