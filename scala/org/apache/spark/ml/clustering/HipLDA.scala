package org.apache.spark.ml.clustering

import org.apache.spark.ml.util.Identifiable
import org.apache.spark.mllib.clustering.{HipOnlineLDAOptimizer, LDA => OldLDA, LocalLDAModel => OldLocalLDAModel}
import org.apache.spark.sql.Dataset

/**
 * ml.clustering.LDA with optimizer = "online" trained on MI355X: the same Params and defaults as
 * [U] spark-mllib 2.4.3 ml.clustering.LDA (k = 10, maxIter = 20, learningOffset = 1024,
 * learningDecay = 0.51, subsamplingRate = 0.05, optimizeDocConcentration = true, seed, docConcentration,
 * topicConcentration), the same fit() construction of the mllib LDA — only the optimizer is
 * HipOnlineLDAOptimizer — and the same result type: an ml LocalLDAModel wrapping the mllib
 * HipLocalLDAModel, so describeTopics, logLikelihood and logPerplexity run on the GPUs that trained it
 * (topicsMatrix, transform and save/load are Spark's own).  setDevices spreads training over several GPUs
 * of this JVM; close the returned model's oldLocalModel (HipLocalLDAModel.close) to release them.
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
    copyValues(new LocalLDAModel(uid, oldModel.vocabSize, oldModel, dataset.sparkSession).setParent(this))
  }
}
