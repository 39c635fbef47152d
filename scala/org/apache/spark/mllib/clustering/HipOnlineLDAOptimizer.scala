package org.apache.spark.mllib.clustering

import org.apache.spark.mllib.linalg.{Matrices, Vector, Vectors}
import org.apache.spark.rdd.RDD

/**
 * OnlineLDAOptimizer whose whole next() — minibatch sampling, the variationalTopicInference E-step,
 * the sufficient statistics, updateLambda / expElogβ and updateAlpha — runs on MI355X through
 * libstc.so (StcNative → jni/stcjni.c → include/stc.h).  Spark's own optimizer is
 * [U] spark-mllib 2.4.3 OnlineLDAOptimizer (TextClustering/build.sbt:10).
 *
 * Drop-in at the reference's optimizer switch (TextClustering/src/main/scala/LDAClustering.scala:40-46):
 * {{{
 *   case "hip-online" => new HipOnlineLDAOptimizer().setMiniBatchFraction(0.05 + 1.0 / actualCorpusSize)
 * }}}
 * Everything else in the file stays: `lda.setOptimizer(optimizer).setK(..)...` (:49-54) and
 * `lda.run(corpus)` (:61), which calls initialize / next × maxIterations / getLDAModel below.
 * LDAOptimizer's three methods are private[clustering]; Scala package-private compiles to public
 * bytecode, so this class works from the application jar in this package.
 *
 * Defaults and setters are OnlineLDAOptimizer's (tau0 1024, kappa 0.51, miniBatchFraction 0.05,
 * optimizeDocConcentration false, gammaShape 100, sampleWithReplacement true); α/η resolution
 * (−1 ⇒ 1/k) happens in stc_lda_create exactly as OnlineLDAOptimizer.initialize does it.  The
 * E-step computes in Double like Breeze (setDtype("f32") selects the fp32 kernels).
 *
 * Layout: the reference runs Spark local[*] (LDATraining.scala:7), one JVM: initialize collects the
 * corpus once into CSR arrays and hands it to a device group (stc_group_*: setDevices(0, 1, …), default
 * device 0), which shards the documents over its GPUs, where they stay for every next().  A group of N
 * devices runs the multi-GPU decomposition — per-device Poisson draws, the stat reduce-scatter, the
 * vocabulary-sliced λ update and its all-gathers — over RCCL when the devices differ.  In a
 * multi-executor deployment each executor instead owns one GPU and a partition: rank 0's
 * StcNative.commUniqueId is broadcast, every executor calls commInit, uploads its partition and
 * passes the global corpus size to ldaSetCorpus.
 *
 * getLDAModel returns a HipLocalLDAModel that takes the group over: its describeTopics,
 * logLikelihood, logPerplexity and topicDistribution(s) run on the GPUs where λ already is.
 */
final class HipOnlineLDAOptimizer extends LDAOptimizer {
  private var tau0: Double = 1024
  private var kappa: Double = 0.51
  private var miniBatchFraction: Double = 0.05
  private var optimizeDocConcentration: Boolean = false
  private var gammaShape: Double = 100
  private var sampleWithReplacement: Boolean = true
  private var dtype: Int = StcNative.F64
  private var devices: Array[Int] = Array(0)

  private var group: Long = 0L
  private var k: Int = 0
  private var vocabSize: Int = 0

  def getTau0: Double = tau0
  def setTau0(tau0: Double): this.type = {
    require(tau0 > 0, s"LDA tau0 must be positive, but was set to $tau0")
    this.tau0 = tau0
    this
  }

  def getKappa: Double = kappa
  def setKappa(kappa: Double): this.type = {
    require(kappa >= 0, s"Online LDA kappa must be nonnegative, but was set to $kappa")
    this.kappa = kappa
    this
  }

  def getMiniBatchFraction: Double = miniBatchFraction
  def setMiniBatchFraction(miniBatchFraction: Double): this.type = {
    require(miniBatchFraction > 0.0 && miniBatchFraction <= 1.0,
      s"Online LDA miniBatchFraction must be in range (0,1], but was set to $miniBatchFraction")
    this.miniBatchFraction = miniBatchFraction
    this
  }

  def getOptimizeDocConcentration: Boolean = optimizeDocConcentration
  def setOptimizeDocConcentration(optimizeDocConcentration: Boolean): this.type = {
    this.optimizeDocConcentration = optimizeDocConcentration
    this
  }

  def getGammaShape: Double = gammaShape
  def setGammaShape(gammaShape: Double): this.type = { this.gammaShape = gammaShape; this }

  def setSampleWithReplacement(b: Boolean): this.type = { this.sampleWithReplacement = b; this }

  /** "f64" (default, Spark's Double arithmetic), "mixed" (the fp32 E-step with its slowly converging
   *  documents re-solved in fp64: the north-star parity bars at ≈ 1.9× the f64 rate) or "f32" */
  def setDtype(d: String): this.type = {
    dtype = d.toLowerCase match {
      case "f64" | "double" => StcNative.F64
      case "mixed" => StcNative.MIXED
      case "f32" | "float" => StcNative.F32
      case other => throw new IllegalArgumentException(s"dtype must be f64, mixed or f32 but got $other")
    }
    this
  }

  def setDevice(d: Int): this.type = setDevices(Array(d))

  /** the GPUs of the group, one document shard each (a repeated id runs several shards on one GPU) */
  def setDevices(ds: Array[Int]): this.type = {
    require(ds.nonEmpty, "at least one device")
    devices = ds.clone()
    this
  }
  def getDevices: Array[Int] = devices.clone()

  override private[clustering] def initialize(docs: RDD[(Long, Vector)], lda: LDA): HipOnlineLDAOptimizer = {
    k = lda.getK
    vocabSize = docs.first()._2.size
    val alpha = lda.getAsymmetricDocConcentration.toArray  // length 1 (−1 ⇒ 1/k) or k, resolved in C
    val rows = docs.sortByKey().values.collect()
    val csr = StcNative.toCsr(rows)
    close()
    group = StcNative.groupCreate(devices, k, vocabSize, alpha, lda.getTopicConcentration, tau0, kappa,
      miniBatchFraction, gammaShape, optimizeDocConcentration, sampleWithReplacement, lda.getSeed, dtype, 0)
    StcNative.groupSetCorpus(group, rows.length, vocabSize, csr(0).asInstanceOf[Array[Long]],
      csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]])
    StcNative.groupInitRandom(group, lda.getSeed)  // λ₀ ~ Gamma(gammaShape, 1/gammaShape)
    this
  }

  /** One OnlineLDAOptimizer.next(): sample → E-step → sstats → (RCCL) → λ / α update, on the GPU. */
  override private[clustering] def next(): HipOnlineLDAOptimizer = {
    StcNative.groupNext(group, null)
    this
  }

  override private[clustering] def getLDAModel(iterationTimes: Array[Double]): LDAModel = {
    val topics = new Array[Double](vocabSize * k)  // k×V row-major = V×k column-major (Matrices.dense)
    StcNative.groupGetTopics(group, topics, StcNative.LAYOUT_KV)
    val alpha = new Array[Double](k)
    StcNative.groupGetAlpha(group, alpha)
    val eta = StcNative.ldaGetEta(StcNative.groupMember(group, 0))
    // the model owns the group from here on (HipLocalLDAModel.close or its finalizer releases it); it
    // infers on the GPUs where λ is, and needs none of the training corpus shards
    StcNative.groupReleaseCorpus(group)
    val model = new HipLocalLDAModel(Matrices.dense(vocabSize, k, topics), Vectors.dense(alpha), eta, gammaShape,
      group)
    group = 0L
    model
  }

  /** The live device group until getLDAModel hands it to the model (0 afterwards). */
  def deviceHandle: Long = group

  /** Releases the device group if no model took it (idempotent). */
  def close(): Unit = {
    if (group != 0L) StcNative.groupDestroy(group)
    group = 0L
  }
}
