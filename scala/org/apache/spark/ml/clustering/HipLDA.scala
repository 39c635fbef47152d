package org.apache.spark.ml.clustering

import org.apache.spark.ml.linalg.Vector
import org.apache.spark.ml.util.Identifiable
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

  /** "f64" (default: Spark's Double E-step) or "f32" */
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
 * E-step's convergence tolerance and γ₀ seeding).  γ₀ of row i of partition p is keyed (seed, p·2^32 + i).
 */
class HipLDAModel private[clustering] (
    uid: String,
    vocabSize: Int,
    private val hip: HipLocalLDAModel,
    sparkSession: SparkSession)
  extends LocalLDAModel(uid, vocabSize, hip, sparkSession) {

  override def transform(dataset: Dataset[_]): DataFrame = {
    if ($(topicDistributionCol).isEmpty) return super.transform(dataset)
    val df = dataset.toDF()
    val outSchema = transformSchema(df.schema, logging = true)
    val featIdx = df.schema.fieldIndex($(featuresCol))
    val key = hip.token
    val cpu = hip.cpuTopicDistributionMethod
    val rows = df.rdd.mapPartitionsWithIndex { (p, it) =>
      val part = it.toArray
      val docs = part.map(r => OldVectors.fromML(r.getAs[Vector](featIdx)))
      val theta = HipLocalLDAModel.topicDistributionsLocal(key, docs, p.toLong << 32).getOrElse(docs.map(cpu))
      part.iterator.zip(theta.iterator).map { case (r, t) => Row.fromSeq(r.toSeq :+ t.asML) }
    }
    df.sparkSession.createDataFrame(rows, outSchema)
  }
}
