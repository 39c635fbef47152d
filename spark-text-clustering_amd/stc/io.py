"""Spark mllib LDA model persistence — the on-disk layout of [U] LocalLDAModel / DistributedLDAModel
``SaveLoadV1_0`` (spark-mllib 2.4.3, TextClustering/build.sbt:10), read and written with pyarrow.
SURVEY.md §8(f) rank 3.

* A model trained here saves as a ``LocalLDAModel`` directory that stock Spark's
  ``LocalLDAModel.load(sc, path)`` reads (the VectorUDT column is marked in the Spark row-schema
  footer key, so ``spark.read.parquet`` hands back Vectors).
* The reference's saved EM models (``TextClustering/src/main/resources/models/*``, written at
  LDAClustering.scala:70 and read at LDALoader.scala:37 with ``DistributedLDAModel.load``) load
  here; ``toLocal`` turns them into a GPU ``LDAModel`` (topicsMatrix = the term vertices' n_wk,
  [U] DistributedLDAModel.topicsMatrix), which is what LDALoader.scala:66/108 then queries.

Layout:

    metadata/part-00000   one JSON line: class, version "1.0", k, vocabSize, docConcentration (k
                          values), topicConcentration, gammaShape (+ iterationTimes: distributed)
    data/                 LocalLDAModel: rows (topic: Vector, index: Int), one per topic — column t
                          of topicsMatrix as a dense vector
    data/globalTopicTotals  DistributedLDAModel: one row (globalTopicTotals: Vector)
    data/topicCounts        (id: Long, topicWeights: Vector); documents id >= 0, terms id = −(v+1)
    data/tokenCounts        (srcId: Long, dstId: Long, tokenCounts: Double) — doc → term edges

Vectors are Spark's VectorUDT struct (type: Byte 0 = sparse / 1 = dense, size: Int, indices:
[Int], values: [Double]).  Host-side file I/O only: no HIP call, nothing on the E-step path.
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np

LOCAL_CLASS = "org.apache.spark.mllib.clustering.LocalLDAModel"
DISTRIBUTED_CLASS = "org.apache.spark.mllib.clustering.DistributedLDAModel"
FORMAT_VERSION = "1.0"
SPARK_ROW_METADATA = "org.apache.spark.sql.parquet.row.metadata"


def _pa():
    import pyarrow as pa
    import pyarrow.parquet as pq

    return pa, pq


def _vector_arrow_type():
    pa, _ = _pa()
    return pa.struct([
        pa.field("type", pa.int8(), nullable=False),
        pa.field("size", pa.int32()),
        pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
        pa.field("values", pa.list_(pa.field("element", pa.float64(), nullable=False))),
    ])


# Spark's JSON for a VectorUDT column (StructField dataType), as DataType.json renders it
_VECTOR_UDT_JSON = {
    "type": "udt",
    "class": "org.apache.spark.mllib.linalg.VectorUDT",
    "pyClass": "pyspark.mllib.linalg.VectorUDT",
    "sqlType": {"type": "struct", "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
        {"name": "indices", "type": {"type": "array", "elementType": "integer", "containsNull": False},
         "nullable": True, "metadata": {}},
        {"name": "values", "type": {"type": "array", "elementType": "double", "containsNull": False},
         "nullable": True, "metadata": {}},
    ]},
}


def _row_metadata(fields):
    """The Spark SQL schema JSON stored under SPARK_ROW_METADATA (fields: [(name, json type, nullable)])."""
    return json.dumps({"type": "struct", "fields": [
        {"name": n, "type": t, "nullable": nb, "metadata": {}} for n, t, nb in fields]}, separators=(",", ":"))


def _dense(v):
    return {"type": 1, "size": None, "indices": None, "values": [float(x) for x in v]}


def _vector_values(vec, size=None):
    """VectorUDT struct (dict) → dense float64 array."""
    if vec["type"] == 1:
        return np.asarray(vec["values"], np.float64)
    out = np.zeros(int(vec["size"] if size is None else size), np.float64)
    out[np.asarray(vec["indices"], np.int64)] = np.asarray(vec["values"], np.float64)
    return out


def _write_table(table, directory, row_meta, part="part-00000"):
    _, pq = _pa()
    os.makedirs(directory, exist_ok=True)
    table = table.replace_schema_metadata({SPARK_ROW_METADATA: row_meta})
    pq.write_table(table, os.path.join(directory, f"{part}.snappy.parquet"), compression="snappy")
    open(os.path.join(directory, "_SUCCESS"), "w").close()


def _read_table(directory):
    pa, pq = _pa()
    files = sorted(glob.glob(os.path.join(directory, "*.parquet")))
    if not files:
        raise FileNotFoundError(f"no parquet part files under {directory}")
    return pa.concat_tables([pq.read_table(f) for f in files])


def _write_metadata(path, meta):
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w", encoding="utf-8") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def read_metadata(path):
    with open(os.path.join(path, "metadata", "part-00000"), encoding="utf-8") as f:
        return json.loads(f.readline())


def _check_overwrite(path, overwrite):
    if os.path.exists(path) and os.listdir(path) and not overwrite:
        raise FileExistsError(f"path {path} already exists (Spark's save refuses to overwrite)")


# ---------------------------------------------------------------------------------------
# LocalLDAModel   [U] LocalLDAModel.SaveLoadV1_0
# ---------------------------------------------------------------------------------------
def save_local(path, topics_matrix, doc_concentration, topic_concentration, gamma_shape=100.0,
               overwrite=False):
    """Write a LocalLDAModel directory: topics_matrix is V×k (Spark's topicsMatrix orientation)."""
    pa, _ = _pa()
    tm = np.asarray(topics_matrix, np.float64)
    if tm.ndim != 2:
        raise ValueError("topics_matrix must be V×k")
    V, k = tm.shape
    alpha = np.broadcast_to(np.asarray(doc_concentration, np.float64), (k,))
    _check_overwrite(path, overwrite)
    _write_metadata(path, {"class": LOCAL_CLASS, "version": FORMAT_VERSION, "k": int(k), "vocabSize": int(V),
                           "docConcentration": [float(a) for a in alpha],
                           "topicConcentration": float(topic_concentration), "gammaShape": float(gamma_shape)})
    topics = pa.array([_dense(tm[:, t]) for t in range(k)], type=_vector_arrow_type())
    index = pa.array(np.arange(k, dtype=np.int32), type=pa.int32())
    table = pa.Table.from_arrays([topics, index], schema=pa.schema([
        pa.field("topic", _vector_arrow_type()), pa.field("index", pa.int32(), nullable=False)]))
    _write_table(table, os.path.join(path, "data"),
                 _row_metadata([("topic", _VECTOR_UDT_JSON, True), ("index", "integer", False)]))


def load_local(path):
    """Read a LocalLDAModel directory → dict(topics V×k, alpha, eta, gamma_shape, k, vocab_size)."""
    meta = read_metadata(path)
    if meta.get("class") != LOCAL_CLASS:
        raise ValueError(f"{path}: class {meta.get('class')!r} is not {LOCAL_CLASS}")
    if meta.get("version") != FORMAT_VERSION:
        raise ValueError(f"{path}: unsupported LocalLDAModel format version {meta.get('version')!r}")
    k, V = int(meta["k"]), int(meta["vocabSize"])
    rows = _read_table(os.path.join(path, "data")).to_pylist()
    if len(rows) != k:
        raise ValueError(f"{path}: {len(rows)} topic rows, metadata says k = {k}")
    tm = np.zeros((V, k), np.float64)
    for r in rows:
        tm[:, int(r["index"])] = _vector_values(r["topic"], V)
    return {"topics": tm, "alpha": np.asarray(meta["docConcentration"], np.float64),
            "eta": float(meta["topicConcentration"]), "gamma_shape": float(meta["gammaShape"]),
            "k": k, "vocab_size": V}


# ---------------------------------------------------------------------------------------
# DistributedLDAModel   [U] DistributedLDAModel.SaveLoadV1_0 (the reference's EM models)
# ---------------------------------------------------------------------------------------
def save_distributed(path, doc_ids, doc_topics, term_topics, edges, doc_concentration, topic_concentration,
                     gamma_shape=100.0, iteration_times=(), overwrite=False):
    """Write a DistributedLDAModel directory (the EM graph): doc_topics D×k (vertex ids doc_ids),
    term_topics V×k (vertex ids −(v+1)), edges = (doc id, term index, token count) arrays."""
    pa, _ = _pa()
    dt = np.asarray(doc_topics, np.float64)
    tt = np.asarray(term_topics, np.float64)
    V, k = tt.shape
    alpha = np.broadcast_to(np.asarray(doc_concentration, np.float64), (k,))
    _check_overwrite(path, overwrite)
    _write_metadata(path, {"class": DISTRIBUTED_CLASS, "version": FORMAT_VERSION, "k": int(k), "vocabSize": int(V),
                           "docConcentration": [float(a) for a in alpha],
                           "topicConcentration": float(topic_concentration),
                           "iterationTimes": [float(x) for x in iteration_times], "gammaShape": float(gamma_shape)})
    vec = _vector_arrow_type()
    totals = tt.sum(axis=0)
    _write_table(pa.Table.from_arrays([pa.array([_dense(totals)], type=vec)], names=["globalTopicTotals"]),
                 os.path.join(path, "data", "globalTopicTotals"),
                 _row_metadata([("globalTopicTotals", _VECTOR_UDT_JSON, True)]))
    ids = np.concatenate([np.asarray(doc_ids, np.int64), -(np.arange(V, dtype=np.int64) + 1)])
    weights = [_dense(r) for r in dt] + [_dense(r) for r in tt]
    _write_table(pa.Table.from_arrays([pa.array(ids, pa.int64()), pa.array(weights, type=vec)],
                                      schema=pa.schema([pa.field("id", pa.int64(), nullable=False),
                                                        pa.field("topicWeights", vec)])),
                 os.path.join(path, "data", "topicCounts"),
                 _row_metadata([("id", "long", False), ("topicWeights", _VECTOR_UDT_JSON, True)]))
    src, term, cnt = (np.asarray(x) for x in edges)
    _write_table(pa.Table.from_arrays([pa.array(src.astype(np.int64)), pa.array(-(term.astype(np.int64) + 1)),
                                       pa.array(cnt.astype(np.float64))],
                                      schema=pa.schema([pa.field("srcId", pa.int64(), nullable=False),
                                                        pa.field("dstId", pa.int64(), nullable=False),
                                                        pa.field("tokenCounts", pa.float64(), nullable=False)])),
                 os.path.join(path, "data", "tokenCounts"),
                 _row_metadata([("srcId", "long", False), ("dstId", "long", False), ("tokenCounts", "double", False)]))


def load_distributed(path):
    """Read a DistributedLDAModel directory → dict(topics V×k = n_wk (toLocal's topicsMatrix),
    global_topic_totals, doc_ids, doc_topics, edges (src, term, count), alpha, eta, gamma_shape,
    iteration_times, k, vocab_size)."""
    meta = read_metadata(path)
    if meta.get("class") != DISTRIBUTED_CLASS:
        raise ValueError(f"{path}: class {meta.get('class')!r} is not {DISTRIBUTED_CLASS}")
    if meta.get("version") != FORMAT_VERSION:
        raise ValueError(f"{path}: unsupported DistributedLDAModel format version {meta.get('version')!r}")
    k, V = int(meta["k"]), int(meta["vocabSize"])
    tc = _read_table(os.path.join(path, "data", "topicCounts"))
    ids = tc.column("id").to_numpy().astype(np.int64)
    weights = tc.column("topicWeights").to_pylist()
    topics = np.zeros((V, k), np.float64)
    seen = np.zeros(V, bool)
    doc_ids, doc_rows = [], []
    for vid, w in zip(ids, weights):
        vals = _vector_values(w, k)
        if vid < 0:
            topics[-(vid + 1)] = vals
            seen[-(vid + 1)] = True
        else:
            doc_ids.append(int(vid))
            doc_rows.append(vals)
    if not seen.all():
        raise ValueError(f"{path}: {int((~seen).sum())} of {V} term vertices missing")
    g = _read_table(os.path.join(path, "data", "globalTopicTotals")).column("globalTopicTotals").to_pylist()
    order = np.argsort(doc_ids, kind="stable")
    tk = _read_table(os.path.join(path, "data", "tokenCounts"))
    src = tk.column("srcId").to_numpy().astype(np.int64)
    term = -(tk.column("dstId").to_numpy().astype(np.int64) + 1)
    return {"topics": topics, "global_topic_totals": _vector_values(g[0], k),
            "doc_ids": np.asarray(doc_ids, np.int64)[order],
            "doc_topics": np.asarray(doc_rows, np.float64).reshape(-1, k)[order],
            "edges": (src, term, tk.column("tokenCounts").to_numpy().astype(np.float64)),
            "alpha": np.asarray(meta["docConcentration"], np.float64), "eta": float(meta["topicConcentration"]),
            "gamma_shape": float(meta.get("gammaShape", 100.0)),
            "iteration_times": np.asarray(meta.get("iterationTimes", []), np.float64), "k": k, "vocab_size": V}
