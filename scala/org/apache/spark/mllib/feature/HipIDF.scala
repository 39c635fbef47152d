package org.apache.spark.mllib.feature

import org.apache.spark.mllib.clustering.StcNative
import org.apache.spark.mllib.linalg.{Vector, Vectors}
import org.apache.spark.rdd.RDD

/**
 * mllib IDF whose document-frequency reduction and idf finalisation run on MI355X (stc_idf_fit:
 * df_j = #docs with value_j > 0, idf_j = df_j ≥ minDocFreq ? ln((m+1)/(df_j+1)) : 0) —
 * [U] spark-mllib 2.4.3 IDF.fit (DocumentFrequencyAggregator).
 *
 * Drop-in at TextClustering/src/main/scala/LDAClustering.scala:177:
 * {{{
 *   val idfVals = new HipIDF(2).fit(tf).idf.toArray       // was: new IDF(2).fit(tf).idf.toArray
 * }}}
 * and, for the reference's ×idf with the 0 → 1e-4 floor (:180-192), `transformWithFloor` keeps the
 * TF·IDF matrix on the GPU (stc_idf_transform with zero_floor = 1e-4).  `fitTransformWithFloor` does
 * both on one upload with the model left on the device (stc_idf_fit_dev → stc_idf_transform_dev): the
 * idf vector never crosses PCIe between the two, and the transform gathers through the model's
 * hot-idf table.
 */
final class HipIDF(val minDocFreq: Int) {
  require(minDocFreq >= 0, s"minDocFreq must be >= 0 but got $minDocFreq")

  def this() = this(0)

  def fit(dataset: RDD[Vector]): IDFModel = {
    val rows = dataset.collect()
    val n = if (rows.isEmpty) 0 else rows.head.size
    val idf = new Array[Double](n)
    if (rows.nonEmpty) {
      val csr = StcNative.toCsr(rows)
      val ctx = StcNative.init(0)
      try {
        val m = StcNative.dcsrUpload(ctx, rows.length, n, csr(0).asInstanceOf[Array[Long]],
          csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], StcNative.F64)
        try StcNative.idfFit(ctx, m, minDocFreq, idf, null)
        finally StcNative.dcsrFree(m)
      } finally StcNative.destroy(ctx)
    }
    new IDFModel(Vectors.dense(idf))
  }

  /** fit + the reference's floored ×idf (LDAClustering.scala:177-192) on one device-resident TF matrix. */
  def fitTransformWithFloor(dataset: RDD[(Long, Vector)], zeroFloor: Double = 1e-4): (IDFModel, RDD[(Long, Vector)]) = {
    val rows = dataset.sortByKey().collect()
    if (rows.isEmpty) return (new IDFModel(Vectors.dense(new Array[Double](0))), dataset)
    val n = rows.head._2.size
    val csr = StcNative.toCsr(rows.map(_._2))
    val idf = new Array[Double](n)
    val ctx = StcNative.init(0)
    val out = try {
      val m = StcNative.dcsrUpload(ctx, rows.length, n, csr(0).asInstanceOf[Array[Long]],
        csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], StcNative.F64)
      try {
        val model = StcNative.idfFitDev(ctx, m, minDocFreq)
        try {
          StcNative.idfTransformDev(ctx, m, model, zeroFloor)
          StcNative.idfGet(ctx, model, n, idf, null)
        } finally StcNative.didfFree(model)
        val ip = csr(0).asInstanceOf[Array[Long]]
        val ix = new Array[Int](ip.last.toInt)
        val vs = new Array[Double](ip.last.toInt)
        StcNative.dcsrDownload(ctx, m, null, ix, vs)
        rows.indices.map { r =>
          val (s, e) = (ip(r).toInt, ip(r + 1).toInt)
          (rows(r)._1, Vectors.sparse(n, ix.slice(s, e), vs.slice(s, e)))
        }
      } finally StcNative.dcsrFree(m)
    } finally StcNative.destroy(ctx)
    (new IDFModel(Vectors.dense(idf)), dataset.sparkContext.parallelize(out, dataset.getNumPartitions))
  }

  /** The reference's TF·IDF (LDAClustering.scala:180-192): values × idf, idf 0 → `zeroFloor`, on the GPU. */
  def transformWithFloor(dataset: RDD[(Long, Vector)], model: IDFModel, zeroFloor: Double = 1e-4): RDD[(Long, Vector)] = {
    val rows = dataset.sortByKey().collect()
    if (rows.isEmpty) return dataset
    val n = rows.head._2.size
    val csr = StcNative.toCsr(rows.map(_._2))
    val ctx = StcNative.init(0)
    val out = try {
      val m = StcNative.dcsrUpload(ctx, rows.length, n, csr(0).asInstanceOf[Array[Long]],
        csr(1).asInstanceOf[Array[Int]], csr(2).asInstanceOf[Array[Double]], StcNative.F64)
      try {
        StcNative.idfTransform(ctx, m, model.idf.toArray, zeroFloor)
        val ip = csr(0).asInstanceOf[Array[Long]]
        val ix = new Array[Int](ip.last.toInt)
        val vs = new Array[Double](ip.last.toInt)
        StcNative.dcsrDownload(ctx, m, null, ix, vs)
        rows.indices.map { r =>
          val (s, e) = (ip(r).toInt, ip(r + 1).toInt)
          (rows(r)._1, Vectors.sparse(n, ix.slice(s, e), vs.slice(s, e)))
        }
      } finally StcNative.dcsrFree(m)
    } finally StcNative.destroy(ctx)
    dataset.sparkContext.parallelize(out, dataset.getNumPartitions)
  }
}
