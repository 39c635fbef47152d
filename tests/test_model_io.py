"""Model persistence (stc.io): LocalLDAModel / DistributedLDAModel in Spark
mllib's SaveLoadV1_0 layout.  CPU tests (pyarrow only).  The reference's own saved EM model is read
when /root/reference is present (this container, never the GPU box) and checked against the
committed fixtures that tests/golden/make_golden.py extracted from the same files."""
import json
import os

import numpy as np
import pytest

from helpers import golden_npz

REF_MODEL = "/root/reference/TextClustering/src/main/resources/models/LdaModel_EN_1591049082850"


def _io():
    from stc import io

    return io


def test_local_model_round_trip(tmp_path):
    io = _io()
    rng = np.random.default_rng(3)
    V, k = 300, 7
    tm = rng.gamma(2.0, 1.0, size=(V, k))
    alpha = rng.uniform(0.05, 1.0, size=k)
    path = str(tmp_path / "m")
    io.save_local(path, tm, alpha, 0.25, gamma_shape=100.0)
    with open(os.path.join(path, "metadata", "part-00000")) as f:
        meta = json.loads(f.readline())
    assert meta["class"] == "org.apache.spark.mllib.clustering.LocalLDAModel" and meta["version"] == "1.0"
    assert (meta["k"], meta["vocabSize"], meta["topicConcentration"], meta["gammaShape"]) == (k, V, 0.25, 100.0)
    m = io.load_local(path)
    assert np.array_equal(m["topics"], tm) and np.array_equal(m["alpha"], alpha)
    assert (m["eta"], m["gamma_shape"], m["k"], m["vocab_size"]) == (0.25, 100.0, k, V)


def test_local_model_parquet_carries_sparks_row_schema(tmp_path):
    """The data parquet holds (topic: VectorUDT, index: int) with Spark's row-schema footer, which
    is what lets spark.read.parquet hand LocalLDAModel.load Vectors."""
    import pyarrow.parquet as pq

    io = _io()
    path = str(tmp_path / "m")
    io.save_local(path, np.ones((5, 2)), [0.5, 0.5], 0.5)
    files = [f for f in os.listdir(os.path.join(path, "data")) if f.endswith(".parquet")]
    t = pq.read_table(os.path.join(path, "data", files[0]))
    assert t.column_names == ["topic", "index"]
    row_meta = json.loads(t.schema.metadata[io.SPARK_ROW_METADATA.encode()])
    f0 = row_meta["fields"][0]
    assert f0["name"] == "topic" and f0["type"]["class"] == "org.apache.spark.mllib.linalg.VectorUDT"
    assert [f["name"] for f in f0["type"]["sqlType"]["fields"]] == ["type", "size", "indices", "values"]
    r = t.to_pylist()[1]
    assert r["index"] == 1 and r["topic"]["type"] == 1 and r["topic"]["values"] == [1.0] * 5


def test_save_refuses_to_overwrite(tmp_path):
    io = _io()
    path = str(tmp_path / "m")
    io.save_local(path, np.ones((4, 2)), [1.0], 1.0)
    with pytest.raises(FileExistsError):
        io.save_local(path, np.ones((4, 2)), [1.0], 1.0)
    io.save_local(path, 2 * np.ones((4, 2)), [1.0], 1.0, overwrite=True)
    assert io.load_local(path)["topics"][0, 0] == 2.0


def test_load_checks_the_model_class(tmp_path):
    io = _io()
    path = str(tmp_path / "m")
    io.save_local(path, np.ones((4, 2)), [1.0], 1.0)
    with pytest.raises(ValueError):
        io.load_distributed(path)


def test_distributed_model_round_trip(tmp_path):
    io = _io()
    rng = np.random.default_rng(4)
    V, k = 40, 3
    doc_ids = np.array([0, 2, 3, 5, 7, 8])  # zipWithIndex ids with gaps (empty docs filtered)
    dt = rng.uniform(0, 10, size=(doc_ids.size, k))
    tt = rng.uniform(0, 10, size=(V, k))
    src = np.repeat(doc_ids, 5)
    term = rng.integers(0, V, src.size)
    cnt = rng.uniform(0.1, 3, src.size)
    path = str(tmp_path / "em")
    io.save_distributed(path, doc_ids, dt, tt, (src, term, cnt), 11.0, 1.1, iteration_times=[0.5, 0.25])
    m = io.load_distributed(path)
    assert np.array_equal(m["topics"], tt) and np.array_equal(m["doc_ids"], doc_ids)
    assert np.array_equal(m["doc_topics"], dt)
    assert np.array_equal(m["global_topic_totals"], tt.sum(axis=0))
    s2, t2, c2 = m["edges"]
    assert np.array_equal(s2, src) and np.array_equal(t2, term) and np.array_equal(c2, cnt)
    assert np.array_equal(m["alpha"], [11.0] * k) and m["eta"] == 1.1
    assert np.array_equal(m["iteration_times"], [0.5, 0.25])


@pytest.mark.skipif(not os.path.isdir(REF_MODEL), reason="reference not present (GPU box)")
def test_reads_the_reference_saved_em_model():
    """LDALoader.scala:37's DistributedLDAModel.load of the reference's own EN model: its term
    vertices equal the committed n_wk fixture, its edges the committed TF·IDF values (F1/F2)."""
    io = _io()
    m = io.load_distributed(REF_MODEL)
    fx = golden_npz("en_topics.npz")
    assert np.array_equal(m["topics"], fx["nwk"])
    assert np.array_equal(m["global_topic_totals"], fx["totals"])
    assert m["k"] == 5 and m["vocab_size"] == 39380 and np.array_equal(m["alpha"], [11.0] * 5)
    assert m["eta"] == 1.1 and m["iteration_times"].size == 50
    idf = golden_npz("en_idf.npz")
    src, term, val = m["edges"]
    o = np.lexsort((term, src))
    assert np.array_equal(val[o], idf["tfidf"])
    assert np.array_equal(np.unique(src), idf["doc_ids"])
