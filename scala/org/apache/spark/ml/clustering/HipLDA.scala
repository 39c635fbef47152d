package org.apache.spark.ml.clustering

import org.apache.spark.ml.linalg.Vector
import org.apache.spark.ml.param.ParamMap
import org.apache.spark.ml.util.{Identifiable, MLReadable, MLReader, MLWriter}
import org.apache.spark.mllib.clustering.{HipLocalLDAModel, HipOnlineLDAOptimizer, LDA => OldLDA, LocalLDAModel => OldLocalLDAModel}
import org.apache.spark.mllib.linalg.{Vectors => OldVectors}
import org.apache.spark.sql.{DataFrame, Dataset, Row, SparkSession}

/**
 * ml.clustering.LDA with optimizer = "online" trained on MI355X: the same Params and defaults as
 * [U] spark-mllib 2.4.3 ml.clustering.LDA (k = 10, maxIter = 20, learningOffset = 1024,
 * learningDecay = 0.51, subsamplingRate = 0.05, optimizeDocConcentration = true, seed, docConcentration,
 * topicConcentration), the same fit() construction of the mllib LDA — only the optimizer is
 * HipOnlineLDAOptimizer — and the same result type: an ml LocalLDAModel wrapping the mllib
 * HipLocalLDAModel, so describeTopics, logLikelihood, logPerplexity and transform (topicDistribution,
 * LDALoader.scala:108's E-step) run on the GPUs that trained it (topicsMatrix and save/load are Spark's
 * own).  setDevices spreads training over several GPUs of this JVM; close the returned model's
 * oldLocalModel (HipLocalLDAModel.close) to release them.
 *
 * {{{
 *   val model = new HipLDA().setK(100).setMaxIter(50).setSeed(1L).setFeaturesCol("features").fit(tfidf)
 * }}}
 */
class HipLDA(override val uid: String) extends LDA(uid) {
  def this() = this(Identifiable.randomUID("hipLDA"))

  /** "f64" (default: Spark's Double E-step), "mixed" (fp32 E-step + fp64 re-solve of the slow documents) or "f32" */
  private var dtype: String = "f64"
  def setDtype(d: String): this.type = { dtype = d; this }

  private var devices: Array[Int] = Array(0)
  def setDevices(ds: Array[Int]): this.type = { devices = ds.clone(); this }

  override def fit(dataset: Dataset[_]): LDAModel = {
    transformSchema(dataset.schema, logging = true)
    require($(optimizer).toLowerCase == "online", s"HipLDA trains the online optimizer only, got ${$(optimizer)}")
    val opt = new HipOnlineLDAOptimizer()
      .setTau0($(learningOffset))
      .setKappa($(learningDecay))
      .setMiniBatchFraction($(subsamplingRate))
      .setOptimizeDocConcentration($(optimizeDocConcentration))
      .setDtype(dtype)
      .setDevices(devices)
    val oldLDA = new OldLDA()
      .setK($(k))
      .setDocConcentration(getOldDocConcentration)
      .setTopicConcentration(getOldTopicConcentration)
      .setMaxIterations($(maxIter))
      .setSeed($(seed))
      .setCheckpointInterval($(checkpointInterval))
      .setOptimizer(opt)
    val oldData = LDA.getOldDataset(dataset, $(featuresCol))
    // the trained HipLocalLDAModel owns the device group; close() frees it only if training failed
    val oldModel = try oldLDA.run(oldData).asInstanceOf[OldLocalLDAModel] finally opt.close()
    val model = oldModel match {
      case h: HipLocalLDAModel => new HipLDAModel(uid, h.vocabSize, h, dataset.sparkSession)
      case m => new LocalLDAModel(uid, m.vocabSize, m, dataset.sparkSession)
    }
    copyValues(model.setParent(this))
  }
}

/**
 * The ml LocalLDAModel HipLDA.fit returns.  transform ([U] ml.clustering.LDAModel.transform: the
 * topicDistributionCol = θ of each row's features) runs one stc_group_topic_distribution call per
 * partition on the GPU group of `hip` instead of Spark's per-row CPU E-step UDF.  A partition evaluated in
 * another JVM, or after the group was released, gets Spark's CPU function (the same result up to the
 * E-step's convergence tolerance and γ₀ seeding); those partitions are counted in `cpuFallbackPartitions`
 * (a Spark accumulator, summed over every transform of this model once its job has run) and logged by the
 * executor that ran them, so a multi-executor deployment can see that the GPU transform did not run there.
 * γ₀ of row i of partition p is keyed (seed, p·2^32 + i).
 *
 * Persistence is Spark's own: `write` saves the model as a plain ml LocalLDAModel (its metadata names
 * LocalLDAModel, so LocalLDAModel.load and PipelineModel.load read it back — ADVICE r5), `copy` keeps
 * this class (pipelines and tuning keep the GPU transform), and HipLDAModel.load delegates to
 * LocalLDAModel.load.
 */
class HipLDAModel private[clustering] (
    uid: String,
    vocabSize: Int,
    private val hip: HipLocalLDAModel,
    sparkSession: SparkSession)
  extends LocalLDAModel(uid, vocabSize, hip, sparkSession) {

  @transient private lazy val fallbacks =
    sparkSession.sparkContext.longAccumulator(s"HipLDAModel($uid).transform CPU-fallback partitions")

  /** Partitions of this model's transforms that ran Spark's CPU E-step (the group was not in their JVM). */
  def cpuFallbackPartitions: Long = fallbacks.value

  override def transform(dataset: Dataset[_]): DataFrame = {
    if ($(topicDistributionCol).isEmpty) return super.transform(dataset)
    val df = dataset.toDF()
    val outSchema = transformSchema(df.schema, logging = true)
    val featIdx = df.schema.fieldIndex($(featuresCol))
    val key = hip.token
    val cpu = hip.cpuTopicDistributionMethod
    val acc = fallbacks
    val id = uid
    val rows = df.rdd.mapPartitionsWithIndex { (p, it) =>
      val part = it.toArray
      val docs = part.map(r => OldVectors.fromML(r.getAs[Vector](featIdx)))
      val theta = HipLocalLDAModel.topicDistributionsLocal(key, docs, p.toLong << 32).getOrElse {
        acc.add(1L)
        System.err.println(s"HipLDAModel($id).transform: partition $p runs Spark's CPU E-step (the GPU group " +
          "is not in this JVM)")
        docs.map(cpu)
      }
      part.iterator.zip(theta.iterator).map { case (r, t) => Row.fromSeq(r.toSeq :+ t.asML) }
    }
    df.sparkSession.createDataFrame(rows, outSchema)
  }

  override def copy(extra: ParamMap): LocalLDAModel = {
    val copied = new HipLDAModel(uid, vocabSize, hip, sparkSession)
    copyValues(copied, extra).setParent(parent).asInstanceOf[LocalLDAModel]
  }

  /** Saved as the plain ml LocalLDAModel it extends (same params, topicsMatrix, α, η, gammaShape). */
  override def write: MLWriter = {
    val plain = new LocalLDAModel(uid, vocabSize, hip, sparkSession)
    copyValues(plain).write
  }
}

object HipLDAModel extends MLReadable[LocalLDAModel] {
  /** A saved HipLDAModel is a LocalLDAModel directory (HipLDAModel.write): read it as one. */
  override def read: MLReader[LocalLDAModel] = LocalLDAModel.read
  override def load(path: String): LocalLDAModel = LocalLDAModel.load(path)
}
