"""GPU: the JNI shim (jni/stcjni.c) end to end on a real device, without a JVM.

tests/jni_stub/mock_env.c in "gpu" mode drives the wrappers against a mock JNIEnv and the real libstc.so on
cuda:0 (no -m gpu test went through the shim):
  * idfGet sizes its checks from the model's own column count (stc_didf_shape): a caller `cols` that
    differs, or a short array, throws IllegalArgumentException instead of overrunning the Java array
    (ADVICE r4); a sized call returns m and df;
  * groupCreate → groupSetTopics → groupTopicDistribution, the call HipLDAModel.transform makes once per
    partition (HipLDA.scala), returns θ equal to the oracle's topicDistribution of the same documents with
    the same γ₀ keys (seed 7, doc_id_base 100 + row) to 1e-10.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "jni_stub")
LIBDIR = os.path.join(ROOT, "spark-text-clustering_amd", "stc")
PREBUILT = os.path.join(STUB, "mock_env")  # __graft_entry__.build() compiles it next to its source


def _mock_exe(tmp_path):
    if os.path.exists(PREBUILT) and os.path.getmtime(PREBUILT) >= os.path.getmtime(os.path.join(STUB, "mock_env.c")):
        return PREBUILT
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not found and no prebuilt mock_env")
    exe = str(tmp_path / "mock_env")
    r = subprocess.run([gcc, "-std=c99", "-O1", "-Wall", "-Wno-unused-parameter", "-I", STUB, "-I",
                        os.path.join(ROOT, "include"), os.path.join(STUB, "mock_env.c"), "-L", LIBDIR, "-lstc",
                        "-Wl,-rpath," + LIBDIR, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_shim_on_the_gpu(tmp_path, oracle):
    out = subprocess.run([_mock_exe(tmp_path), "gpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = {}
    for line in out.stdout.strip().splitlines():
        f = line.split("\t")
        rows[f[0]] = f[1:]
    ok = ["-", "-"]
    for name in ("init", "dcsrUpload", "idfFitDev", "idfGet_sized", "groupCreate", "groupSetTopics",
                 "groupTopicDistribution"):
        assert rows[name] == ok, (name, rows[name])
    iae = "java/lang/IllegalArgumentException"
    assert rows["idfGet_wrong_cols"] == [iae, "idfGet: cols = 9, the model has 10 columns"]
    assert rows["idfGet_short_idf"] == [iae, "idfGet idfOut: the Java array has 9 elements, the call needs 10"]
    m, dfs = rows["idfGet_result"]
    assert int(m) == 3 and [int(x) for x in dfs.split()] == [1, 1, 3, 1]  # df of terms 0, 1, 3, 9
    assert int(rows["transport"][0]) == 0  # one member: no collectives
    # θ against the oracle: λ as mock_env sets it (V×k, element j = 0.5 + 0.37·((7j) mod 11)), α = η = 1/k
    V, k = 10, 3
    lam = np.array([0.5 + 0.37 * ((j * 7) % 11) for j in range(V * k)]).reshape(V, k)
    alpha, _ = oracle.resolve_alpha_eta(k)
    docs = [([0, 3], [2.0, 1.0]), ([3], [4.0]), ([1, 3, 9], [1.0, 2.0, 5.0])]
    theta = np.array([float(x) for x in rows["theta"]]).reshape(3, k)
    for r, (ids, cts) in enumerate(docs):
        g0 = oracle.gamma_init(7, 100 + r, k)
        want = oracle.topic_distribution(np.array(ids), np.array(cts), lam, alpha, g0)
        np.testing.assert_allclose(theta[r], want, rtol=1e-10, atol=1e-14)


def _train_through_shim(tmp_path, corpus, devices, k, steps, seed, frac, env=None):
    """mock_env gpu_train: HipOnlineLDAOptimizer's JNI calls over `corpus` (see mock_env.c)"""
    import struct

    inp, outp = tmp_path / "train.in", tmp_path / "train.out"
    with open(inp, "wb") as f:
        f.write(struct.pack("<q", len(devices)))
        f.write(np.asarray(devices, "<i8").tobytes())
        f.write(struct.pack("<qqqqqd", corpus.num_rows, corpus.num_cols, k, steps, seed, frac))
        f.write(np.asarray(corpus.indptr, "<i8").tobytes())
        f.write(np.asarray(corpus.indices, "<i4").tobytes())
        f.write(np.asarray(corpus.values, "<f8").tobytes())
    run_env = dict(os.environ, **(env or {}))
    out = subprocess.run([_mock_exe(tmp_path), "gpu_train", str(inp), str(outp)], capture_output=True, text=True,
                         timeout=240, env=run_env)
    assert out.returncode == 0, out.stdout + out.stderr
    # (RCCL prints its version banner to stdout: only the mock's three-field report lines)
    calls = [line.split("\t") for line in out.stdout.strip().splitlines() if line.count("\t") == 2]
    for c in calls:
        assert c[1:] == ["-", "-"], c  # no Java exception from any wrapper
    V = corpus.num_cols
    b = np.fromfile(outp, np.uint8)
    off = 0

    def take(n, dt):
        nonlocal off
        a = np.frombuffer(b[off:off + n * np.dtype(dt).itemsize].tobytes(), dt)
        off += n * np.dtype(dt).itemsize
        return a

    res = dict(lam_kv=take(V * k, "<f8").reshape(k, V), alpha=take(k, "<f8"), eta=take(1, "<f8")[0],
               iteration=int(take(1, "<f8")[0]), stats=take(steps * 7, "<f8").reshape(steps, 7),
               didx=take(k * 10, "<i4").reshape(k, 10), dw=take(k * 10, "<f8").reshape(k, 10),
               bound=take(4, "<f8"), transport=int(take(1, "<f8")[0]), calls=[c[0] for c in calls])
    assert off == b.size
    return res


@pytest.mark.parametrize("devices,rccl", [([0, 0], "0"), ([0], "1")])
def test_shim_training_path_on_the_gpu(tmp_path, oracle, devices, rccl):
    """the JVM drop-in's TRAINING path through the JNI shim on the device — groupCreate →
    groupSetCorpus → groupInitRandom → groupNext × 10 → groupGetTopics / groupGetAlpha / ldaGetEta →
    groupReleaseCorpus → groupDescribe / groupBound → groupDestroy, in HipOnlineLDAOptimizer.scala:105-139's
    and HipLocalLDAModel's order — once over two members on the one GPU (in-process transport) and once as a
    one-device RCCL group (STC_GROUP_RCCL=1).  λ / α within 1e-9 of the oracle replaying the same
    device-sampled membership from the same λ₀ (oracle.init_lambda: the counter RNG groupInitRandom
    draws), describeTopics and the bound against the oracle's on the trained model."""
    import stc
    from helpers import random_corpus
    from test_gpu_comm import _members
    from test_gpu_group import _shard_rows

    rng = np.random.default_rng(300)
    D, V, k, steps, seed, frac = 300, 800, 8, 10, 77, 0.1
    corpus = random_corpus(rng, D, V, 1, 40, empty_every=13)
    r = _train_through_shim(tmp_path, corpus, devices, k, steps, seed, frac, {"STC_GROUP_RCCL": rccl})
    assert r["transport"] == (1 if len(devices) > 1 else 2)  # IN_PROCESS / RCCL
    assert r["calls"].count("groupNext") == steps
    members = len(devices)
    r0 = _shard_rows(corpus.indptr, members)
    alpha0, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=oracle.init_lambda(seed, V, k).T.copy(), alpha=alpha0, eta=eta, corpus_size=D,
                               mini_batch_fraction=frac, optimize_doc_concentration=True)
    sizes = []
    for draw in range(1, steps + 1):
        it = st.iteration + 1
        docs, g0 = [], []
        for q in range(members):
            lo, hi = r0[q], r0[q + 1]
            ip = corpus.indptr[lo:hi + 1] - corpus.indptr[lo]
            for pos, dl in enumerate(_members(ip, frac, seed, draw, q, oracle)):
                docs.append(corpus.row(lo + dl))
                g0.append(oracle.gamma_init(seed, oracle.train_doc_key(it, q, pos), k))
        sizes.append(len(docs))
        if docs:
            oracle.submit_minibatch(st, docs, g0)
    assert r["iteration"] == st.iteration > 0
    assert [int(x) for x in r["stats"][:, 0]] == sizes  # batch docs per next(), through the stats array
    lam = r["lam_kv"].T  # V×k
    rel = np.max(np.abs(lam - st.lam.T) / st.lam.T)
    assert rel < 1e-9, rel
    np.testing.assert_allclose(r["alpha"], st.alpha, rtol=1e-9)
    assert r["eta"] == eta
    oi, ow = oracle.describe_topics(st.lam.T, 10)
    assert np.array_equal(r["didx"], oi)
    np.testing.assert_allclose(r["dw"], ow, rtol=1e-8)
    docs = [corpus.row(i) for i in range(D)]
    want, _, _ = oracle.log_likelihood_bound(docs, [oracle.gamma_init(9, i, k) for i in range(D)], st.lam.T,
                                             st.alpha, eta)
    np.testing.assert_allclose(r["bound"][0], want, rtol=1e-8)
    assert r["bound"][3] == float(corpus.values.sum())
