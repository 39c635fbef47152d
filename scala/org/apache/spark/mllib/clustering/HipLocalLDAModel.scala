package org.apache.spark.mllib.clustering

import org.apache.spark.mllib.linalg.{Matrix, Vector, Vectors}
import org.apache.spark.rdd.RDD

/**
 * The LocalLDAModel HipOnlineLDAOptimizer.getLDAModel returns: a stock [U] spark-mllib 2.4.3
 * LocalLDAModel (topicsMatrix, save/load and serialisation are Spark's own) whose inference calls run on
 * the GPU group that trained it, where λ is still resident:
 *
 *   describeTopics      → stc_group_describe   (the reference's LDAClustering.scala describeTopics call)
 *   logLikelihood       → stc_group_bound      (LocalLDAModel.logLikelihoodBound: corpus part + topics part)
 *   logPerplexity       → stc_group_bound      (−bound / token count, one device pass instead of two RDD jobs)
 *   topicDistribution(s)→ stc_group_topic_distribution (zeros for empty documents, as Spark)
 *   getTopicDistributionMethod (the row function of ml LocalLDAModel.transform)
 *                       → stc_group_topic_distribution, via the JVM-local registry (token)
 *
 * The documents of an RDD call are collected to the driver (the reference runs local[*], one JVM:
 * LDATraining.scala:7) and sharded over the group's devices.  γ₀ of document i (its position in the
 * collected RDD) comes from the counter RNG keyed (getSeed, i) — a seeded draw from Spark's
 * Gamma(gammaShape, 1/gammaShape), not Breeze's generator stream, so results equal Spark's to the
 * E-step's convergence tolerance, not bit for bit (DESIGN.md §3).
 *
 * The group handle is transient: a deserialised copy, or one after close(), has none and every method
 * falls back to Spark's CPU implementation.  A group handle is not thread-safe, so every call on it is
 * serialised by the model's lock (describeTopics / logLikelihood / topicDistribution may be called from
 * several threads on a shared model); the finalizer releases the group of a model nobody closed.
 */
final class HipLocalLDAModel private[clustering] (
    topicsM: Matrix,
    alphaV: Vector,
    etaV: Double,
    shape: Double,
    @transient private var group: Long)
  extends LocalLDAModel(topicsM, alphaV, etaV, shape) {

  @transient private lazy val lock = new Object

  /**
   * This model's key in the JVM-wide registry (serialised with the model and with the closures below): a
   * task deserialised in the JVM that holds the group (Spark local[*], the reference's deployment,
   * LDATraining.scala:7) finds the live model under it and runs on its GPUs; any other JVM finds nothing
   * and runs Spark's CPU E-step.  The raw group pointer itself never leaves the driver.
   */
  private[clustering] val token: String = java.util.UUID.randomUUID().toString
  HipLocalLDAModel.register(this)

  /** true while the model's λ is resident on the GPU group */
  def onDevice: Boolean = lock.synchronized(group != 0L)

  /** Releases the GPU group (the model keeps its host copy of λ and falls back to the CPU). */
  def close(): Unit = lock.synchronized {
    if (group != 0L) StcNative.groupDestroy(group)
    group = 0L
    HipLocalLDAModel.unregister(token)
  }

  /**
   * θ = γ/Σγ of every document on this model's GPU group (one stc_group_topic_distribution call for the
   * batch, documents sharded over the devices), or None when the group was released.  docIdBase keys γ₀.
   */
  private[clustering] def deviceTopicDistributions(docs: Array[Vector], docIdBase: Long): Option[Array[Vector]] =
    lock.synchronized {
      if (group == 0L) None
      else {
        docs.foreach(v => require(v.size == vocabSize, s"document of size ${v.size}, the model has $vocabSize terms"))
        val csr = StcNative.toCsr(docs)
        val out = new Array[Double](docs.length * k)
        StcNative.groupTopicDistribution(group, docs.length, vocabSize, csr(0).asInstanceOf[Array[Long]],
          csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], getSeed, docIdBase, null, out)
        Some(Array.tabulate(docs.length)(i => Vectors.dense(out.slice(i * k, (i + 1) * k))))
      }
    }

  /**
   * [U] LocalLDAModel.getTopicDistributionMethod: the per-row function ml.clustering.LocalLDAModel.transform
   * wraps in its UDF (so the stock ml transform of a model wrapping this one reaches the GPU as well, one
   * document per call — HipLDAModel.transform batches a whole partition per call instead).  The closure
   * carries the registry token and Spark's own CPU function as the fallback for another JVM.
   */
  override private[spark] def getTopicDistributionMethod: Vector => Vector = {
    val key = token
    val cpu = cpuTopicDistributionMethod
    (v: Vector) => HipLocalLDAModel.topicDistributionsLocal(key, Array(v), 0L).map(_(0)).getOrElse(cpu(v))
  }

  /** Spark's own CPU row function (the fallback the closures above carry to other JVMs) */
  private[spark] def cpuTopicDistributionMethod: Vector => Vector = super.getTopicDistributionMethod

  override protected def finalize(): Unit = {
    try close() finally super.finalize()
  }

  /** f(group) under the lock, or the CPU fallback when the model holds no group */
  private def onGroup[T](cpu: => T)(f: Long => T): T = lock.synchronized {
    if (group == 0L) cpu else f(group)
  }

  override def describeTopics(maxTermsPerTopic: Int): Array[(Array[Int], Array[Double])] =
    onGroup(super.describeTopics(maxTermsPerTopic)) { g =>
      val n = math.max(0, math.min(maxTermsPerTopic, vocabSize))
      val idx = new Array[Int](k * n)
      val w = new Array[Double](k * n)
      StcNative.groupDescribe(g, maxTermsPerTopic, idx, w)
      Array.tabulate(k)(t => (idx.slice(t * n, (t + 1) * n), w.slice(t * n, (t + 1) * n)))
    }

  private def collectCsr(documents: RDD[(Long, Vector)]): (Array[Long], Array[Vector], Array[AnyRef]) = {
    val docs = documents.collect()
    val rows = docs.map(_._2)
    rows.foreach(v => require(v.size == vocabSize, s"document of size ${v.size}, the model has $vocabSize terms"))
    (docs.map(_._1), rows, StcNative.toCsr(rows))
  }

  /** {bound, corpusPart, topicsPart, tokenCount} of the documents on the GPU group g */
  private def deviceBound(g: Long, documents: RDD[(Long, Vector)]): Array[Double] = {
    val (_, rows, csr) = collectCsr(documents)
    StcNative.groupBound(g, rows.length, vocabSize, csr(0).asInstanceOf[Array[Long]],
      csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], getSeed, 0L, null)
  }

  override def logLikelihood(documents: RDD[(Long, Vector)]): Double =
    onGroup(super.logLikelihood(documents))(g => deviceBound(g, documents)(0))

  override def logPerplexity(documents: RDD[(Long, Vector)]): Double =
    onGroup(super.logPerplexity(documents)) { g =>
      val r = deviceBound(g, documents)
      -r(0) / r(3)
    }

  override def topicDistributions(documents: RDD[(Long, Vector)]): RDD[(Long, Vector)] =
    onGroup(super.topicDistributions(documents)) { g =>
      val (ids, rows, csr) = collectCsr(documents)
      val out = new Array[Double](rows.length * k)
      StcNative.groupTopicDistribution(g, rows.length, vocabSize, csr(0).asInstanceOf[Array[Long]],
        csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], getSeed, 0L, null, out)
      val theta = Array.tabulate(rows.length)(i => (ids(i), Vectors.dense(out.slice(i * k, (i + 1) * k))))
      documents.sparkContext.parallelize(theta, math.max(1, documents.getNumPartitions))
    }

  override def topicDistribution(document: Vector): Vector =
    onGroup(super.topicDistribution(document)) { g =>
      require(document.size == vocabSize, s"document of size ${document.size}, the model has $vocabSize terms")
      val csr = StcNative.toCsr(Array(document))
      val out = new Array[Double](k)
      StcNative.groupTopicDistribution(g, 1, vocabSize, csr(0).asInstanceOf[Array[Long]],
        csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], getSeed, 0L, null, out)
      Vectors.dense(out)
    }
}

object HipLocalLDAModel {
  // the JVM's models that hold a GPU group, by token (weak: a model nobody references can still be collected)
  private val live = new java.util.concurrent.ConcurrentHashMap[String, java.lang.ref.WeakReference[HipLocalLDAModel]]()

  private def register(m: HipLocalLDAModel): Unit = live.put(m.token, new java.lang.ref.WeakReference(m))
  private def unregister(token: String): Unit = live.remove(token)

  /**
   * θ of `docs` on the GPU group of the model registered under `token` in THIS JVM, or None (no such model
   * here, or its group was released): the caller then uses Spark's CPU E-step.
   */
  private[spark] def topicDistributionsLocal(token: String, docs: Array[Vector], docIdBase: Long): Option[Array[Vector]] = {
    val ref = live.get(token)
    val m = if (ref == null) null else ref.get()
    if (m == null) None else m.deviceTopicDistributions(docs, docIdBase)
  }

  /**
   * A GPU copy of an already trained model, e.g. the reference's LDALoader.scala:108
   * `LDATrainedModel.toLocal.topicDistribution(v)` becomes
   * `HipLocalLDAModel.fromLocal(LDATrainedModel.toLocal).topicDistribution(v)`.  λ (topicsMatrix), α, η
   * and gammaShape are the model's; the group holds no corpus (inference only).
   */
  def fromLocal(m: LocalLDAModel, devices: Array[Int] = Array(0), dtype: Int = StcNative.F64): HipLocalLDAModel = {
    val g = StcNative.groupCreate(devices, m.k, m.vocabSize, m.docConcentration.toArray, m.topicConcentration,
      1024, 0.51, 0.05, m.gammaShape, false, true, m.getSeed, dtype, 0)
    try {
      // topicsMatrix is V×k column-major = k×V row-major (LAYOUT_KV)
      StcNative.groupSetTopics(g, m.topicsMatrix.toArray, StcNative.LAYOUT_KV)
    } catch {
      case e: Throwable =>
        StcNative.groupDestroy(g)
        throw e
    }
    val h = new HipLocalLDAModel(m.topicsMatrix, m.docConcentration, m.topicConcentration, m.gammaShape, g)
    h.setSeed(m.getSeed)
    h
  }
}
