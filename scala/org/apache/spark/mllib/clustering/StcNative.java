package org.apache.spark.mllib.clustering;

/**
 * JNI declarations of libstc.so (include/stc.h) — one native method per C entry point, implemented
 * by jni/stcjni.c (libstcjni.so, which links libstc.so).  Handles (stc_ctx*, stc_dcsr*, stc_lda*) are
 * longs; a non-zero status surfaces as IllegalArgumentException (STC_ERR_INVALID_ARG) or
 * IllegalStateException with the library's message.  Callers: HipOnlineLDAOptimizer (the
 * LDAClustering.scala:40-46 optimizer switch), mllib.feature.HipIDF (LDAClustering.scala:177), and
 * the Spark-ML wrappers HipHashingTF / HipLDA.
 */
public final class StcNative {
  static {
    System.loadLibrary("stcjni");
  }

  private StcNative() {}

  public static final int F32 = 0, F64 = 1;
  /** LDA dtype only: the fp32 E-step with the documents past 500 fp32 iterations re-solved in fp64 (stc.h STC_MIXED) */
  public static final int MIXED = 2;
  public static final int HASH_STANDARD = 0, HASH_SPARK24 = 1;
  public static final int LAYOUT_VK = 0, LAYOUT_KV = 1;

  // ---- library / device
  public static native String lastError();
  public static native int abiVersion();
  public static native int deviceCount();
  public static native long init(int device);
  public static native void destroy(long ctx);
  public static native void synchronize(long ctx);

  // ---- RCCL (one process per GPU: rank 0's id is broadcast by the driver)
  public static native byte[] commUniqueId();
  public static native void commInit(long ctx, byte[] id, int nRanks, int rank);
  public static native void commAllreduceF64(long ctx, double[] inout);

  // ---- device CSR (rows = documents)
  public static native long dcsrUpload(long ctx, long rows, long cols, long[] indptr, int[] indices,
                                       double[] values, int valueDtype);
  /** {rows, cols, nnz} */
  public static native long[] dcsrShape(long dcsr);
  public static native void dcsrDownload(long ctx, long dcsr, long[] indptr, int[] indices, double[] values);
  public static native void dcsrFree(long dcsr);

  // ---- HashingTF: token t = utf8[tokOff[t], tokOff[t+1]), doc d = tokens [docOff[d], docOff[d+1])
  public static native long hashingTfDev(long ctx, byte[] utf8, long[] tokOff, long[] docOff, int numFeatures,
                                         boolean binary, int hashVariant, int valueDtype);
  public static native void hashingTf(long ctx, byte[] utf8, long[] tokOff, long[] docOff, int numFeatures,
                                      boolean binary, int hashVariant, long[] indptrOut, int[] indicesOut,
                                      double[] valuesOut);
  public static native void hashTokens(long ctx, byte[] utf8, long[] tokOff, int numFeatures, int hashVariant,
                                       int[] idxOut);
  /** tokens kept on the GPU between calls (stc_tokens_upload / stc_hashing_tf_tokens) */
  public static native long tokensUpload(long ctx, byte[] utf8, long[] tokOff, long[] docOff);
  public static native void tokensFree(long tokens);
  public static native long hashingTfTokens(long ctx, long tokens, int numFeatures, boolean binary, int hashVariant,
                                            int valueDtype);

  // ---- Tokenizer (ml.feature.Tokenizer: toLowerCase.split("\\s")); returns {nOutBytes, nTok}.
  // utf8Out holds text.length * 3 / 2 bytes (Java lower-cases a few 2-byte characters to 3 bytes)
  public static native long[] tokenize(long ctx, byte[] text, long[] textOff, byte[] utf8Out, long[] tokOffOut,
                                       long[] docOffOut);
  public static native long tokenizeHashingTfDev(long ctx, byte[] text, long[] textOff, int numFeatures,
                                                 boolean binary, int hashVariant, int valueDtype);

  // ---- IDF: returns m (documents, summed over ranks)
  public static native long idfFit(long ctx, long dcsr, long minDocFreq, double[] idfOut, long[] dfOut);
  public static native void idfTransform(long ctx, long dcsr, double[] idf, double zeroFloor);
  // the IDF model kept on the device (a handle); idfGet copies idf / df out (either may be null), returns m
  public static native long idfFitDev(long ctx, long dcsr, long minDocFreq);
  public static native long idfGet(long ctx, long model, long cols, double[] idfOut, long[] dfOut);
  public static native void idfTransformDev(long ctx, long dcsr, long model, double zeroFloor);
  // {numFeatures, m} of a device IDF model (idfGet's cols must equal numFeatures)
  public static native long[] didfShape(long model);
  public static native void didfFree(long model);

  // ---- online LDA (alpha null ⇒ −1 ⇒ 1/k; eta −1 ⇒ 1/k)
  public static native long ldaCreate(long ctx, int k, long vocabSize, double[] alpha, double eta, double tau0,
                                      double kappa, double miniBatchFraction, double gammaShape,
                                      boolean optimizeDocConcentration, boolean sampleWithReplacement, long seed,
                                      int dtype, int maxInnerIter);
  public static native void ldaDestroy(long lda);
  public static native void ldaSetCorpus(long lda, long dcsr, long corpusSizeTotal);
  public static native void ldaInitRandom(long lda, long seed);
  public static native void ldaSetTopics(long lda, double[] topics, int layout);
  public static native void ldaGetTopics(long lda, double[] out, int layout);
  public static native void ldaSetAlpha(long lda, double[] alpha);
  public static native void ldaGetAlpha(long lda, double[] out);
  public static native double ldaGetEta(long lda);
  public static native long ldaGetIteration(long lda);
  /** {k, vocabSize} of the handle */
  public static native long[] ldaShape(long lda);
  /** stats (nullable, 7): batchDocs, nonemptyDocs, batchEntries, innerIters, innerItersMax, capHits, rho */
  public static native void ldaStep(long lda, long[] batchDocIds, double[] gamma0, double[] stats);
  public static native void ldaNext(long lda, double[] stats);
  public static native void ldaEstep(long lda, long[] batchDocIds, double[] gamma0, double[] gammaOut,
                                     double[] statOut, int[] itersOut);
  /** {bound, corpusPart, topicsPart, tokenCount} */
  public static native double[] ldaBound(long lda, long dcsr, long gammaSeed, long docIdBase, double[] gamma0);
  public static native void ldaTopicDistribution(long lda, long dcsr, long gammaSeed, long docIdBase,
                                                 double[] gamma0, double[] out);
  public static native void ldaDescribe(long lda, int maxTerms, int[] idxOut, double[] weightOut);
  public static native void ldaEnableTiming(long lda, boolean on);
  public static native void ldaCounters(long lda, long[] out4);
  public static native long ldaPhaseTimes(long lda, double[] msOut5);
  /** E-step launches per kernel family (stc.h enum stc_kernel_count), 12 words */
  public static native void ldaKernelCounts(long lda, long[] out12);

  // ---- host helpers (pure Java): Spark vectors → CSR arrays
  /** CSR of sparse or dense rows: {indptr long[n+1], indices int[nnz], values double[nnz]} */
  public static Object[] toCsr(org.apache.spark.mllib.linalg.Vector[] rows) {
    org.apache.spark.mllib.linalg.SparseVector[] sp = new org.apache.spark.mllib.linalg.SparseVector[rows.length];
    long[] indptr = new long[rows.length + 1];
    int nnz = 0;
    for (int i = 0; i < rows.length; ++i) {
      sp[i] = rows[i].toSparse();  // sorted indices, explicit zeros dropped
      nnz += sp[i].indices().length;
      indptr[i + 1] = nnz;
    }
    int[] indices = new int[nnz];
    double[] values = new double[nnz];
    int p = 0;
    for (org.apache.spark.mllib.linalg.SparseVector s : sp) {
      System.arraycopy(s.indices(), 0, indices, p, s.indices().length);
      System.arraycopy(s.values(), 0, values, p, s.values().length);
      p += s.indices().length;
    }
    return new Object[] {indptr, indices, values};
  }

  // ---- one process, N devices (stc_group): the multi-GPU form of the drop-in inside one JVM ----------
  public static native long groupCreate(int[] deviceIds, int k, long vocabSize, double[] alpha, double eta,
                                        double tau0, double kappa, double miniBatchFraction, double gammaShape,
                                        boolean optimizeAlpha, boolean withReplacement, long seed, int dtype,
                                        int maxInnerIter);
  public static native void groupDestroy(long group);
  public static native int groupSize(long group);
  // how the group's collectives travel: 0 none (one member), 1 in-process (one device repeated), 2 RCCL
  public static native int groupTransport(long group);
  public static native long groupMember(long group, int i);
  public static native void groupSetCorpus(long group, long rows, long cols, long[] indptr, int[] indices,
                                           double[] values);
  public static native void groupReleaseCorpus(long group);
  public static native void groupInitRandom(long group, long seed);
  public static native void groupSynchronize(long group);
  public static native void groupSetTopics(long group, double[] topics, int layout);
  public static native void groupGetTopics(long group, double[] out, int layout);
  public static native void groupGetAlpha(long group, double[] out);
  public static native long groupGetIteration(long group);
  public static native void groupNext(long group, double[] stats);
  public static native void groupStep(long group, long[] batchDocIds, double[] gamma0, double[] stats);
  public static native void groupDescribe(long group, int maxTerms, int[] idxOut, double[] weightOut);
  /** {bound, corpusPart, topicsPart, tokenCount} */
  public static native double[] groupBound(long group, long rows, long cols, long[] indptr, int[] indices,
                                           double[] values, long gammaSeed, long docIdBase, double[] gamma0);
  public static native void groupTopicDistribution(long group, long rows, long cols, long[] indptr, int[] indices,
                                                   double[] values, long gammaSeed, long docIdBase,
                                                   double[] gamma0, double[] out);
}
