package org.apache.spark.ml.feature

import java.nio.charset.StandardCharsets

import org.apache.spark.ml.Transformer
import org.apache.spark.ml.linalg.{SQLDataTypes, Vectors}
import org.apache.spark.ml.param.{BooleanParam, IntParam, ParamMap, ParamValidators}
import org.apache.spark.ml.param.shared.{HasInputCol, HasOutputCol}
import org.apache.spark.ml.util.Identifiable
import org.apache.spark.mllib.clustering.StcNative
import org.apache.spark.sql.{DataFrame, Dataset, Row}
import org.apache.spark.sql.types.{ArrayType, StringType, StructField, StructType}

/**
 * ml.feature.HashingTF on MI355X: per partition, the tokens go to the GPU as one UTF-8 blob and come
 * back as the sorted sparse term-frequency vectors (stc_hashing_tf: murmur3_x86_32 with seed 42,
 * nonNegativeMod(numFeatures), counts or binary) — bit-exact with [U] spark-mllib 2.4.3
 * HashingTF.transform, whose Murmur3_x86_32.hashUnsafeBytes tail (hashVariant 1) is the default here.
 * Same params as Spark's (numFeatures = 2^18, binary = false, inputCol, outputCol).  The slot in the
 * reference is the vocabulary counting at LDAClustering.scala:154-167.
 */
class HipHashingTF(override val uid: String) extends Transformer with HasInputCol with HasOutputCol {
  def this() = this(Identifiable.randomUID("hipHashingTF"))

  val numFeatures = new IntParam(this, "numFeatures", "number of features (> 0)", ParamValidators.gt(0))
  val binary = new BooleanParam(this, "binary", "If true, all non zero counts are set to 1.")
  /** 1 = Spark 2.4.x hashUnsafeBytes (default), 0 = standard MurmurHash3_x86_32 tail (Spark 3.x) */
  val hashVariant = new IntParam(this, "hashVariant", "murmur3 tail variant", ParamValidators.inArray(Array(0, 1)))
  /** GPU device index used by the executors */
  val device = new IntParam(this, "device", "GPU device index", ParamValidators.gtEq(0))
  setDefault(numFeatures -> (1 << 18), binary -> false, hashVariant -> StcNative.HASH_SPARK24, device -> 0)

  def setInputCol(value: String): this.type = set(inputCol, value)
  def setOutputCol(value: String): this.type = set(outputCol, value)
  def setNumFeatures(value: Int): this.type = set(numFeatures, value)
  def getNumFeatures: Int = $(numFeatures)
  def setBinary(value: Boolean): this.type = set(binary, value)
  def getBinary: Boolean = $(binary)

  override def transform(dataset: Dataset[_]): DataFrame = {
    val outSchema = transformSchema(dataset.schema)
    val inIdx = dataset.schema.fieldIndex($(inputCol))
    val (nf, bin, hv, dev) = ($(numFeatures), $(binary), $(hashVariant), $(device))
    val rows = dataset.toDF().rdd.mapPartitions { it =>
      val part = it.toArray
      if (part.isEmpty) Iterator.empty
      else {
        val toks = part.map(_.getSeq[String](inIdx))
        val bytes = toks.flatMap(_.map(_.getBytes(StandardCharsets.UTF_8)))
        val tokOff = bytes.scanLeft(0L)(_ + _.length)
        val docOff = toks.scanLeft(0L)(_ + _.length)
        val blob = new Array[Byte](tokOff.last.toInt)
        var p = 0
        bytes.foreach { b => System.arraycopy(b, 0, blob, p, b.length); p += b.length }
        val indptr = new Array[Long](part.length + 1)
        val idx = new Array[Int](bytes.length)
        val vals = new Array[Double](bytes.length)
        val ctx = StcNative.init(dev)
        try StcNative.hashingTf(ctx, blob, tokOff, docOff, nf, bin, hv, indptr, idx, vals)
        finally StcNative.destroy(ctx)
        part.indices.iterator.map { d =>
          val (s, e) = (indptr(d).toInt, indptr(d + 1).toInt)
          Row.fromSeq(part(d).toSeq :+ Vectors.sparse(nf, idx.slice(s, e), vals.slice(s, e)))
        }
      }
    }
    dataset.sparkSession.createDataFrame(rows, outSchema)
  }

  override def transformSchema(schema: StructType): StructType = {
    val t = schema($(inputCol)).dataType
    require(t.isInstanceOf[ArrayType] && t.asInstanceOf[ArrayType].elementType == StringType,
      s"The input column must be ArrayType(StringType), but got $t.")
    require(!schema.fieldNames.contains($(outputCol)), s"Output column ${$(outputCol)} already exists.")
    StructType(schema.fields :+ StructField($(outputCol), SQLDataTypes.VectorType, nullable = false))
  }

  override def copy(extra: ParamMap): HipHashingTF = defaultCopy(extra)
}
