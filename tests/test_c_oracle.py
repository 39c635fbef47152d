"""CPU: the C/OpenMP oracle (bench cpu_baseline) agrees with the fixture-pinned NumPy oracle."""
import numpy as np
import pytest

from helpers import golden_json, golden_npz, random_corpus


@pytest.fixture(scope="module")
def co():
    from oracle import c_oracle

    if not c_oracle.available():
        pytest.skip("oracle/_build/liblda_oracle.so not built (make -C oracle)")
    return c_oracle


def test_c_oracle_matches_numpy_oracle(co, oracle):
    rng = np.random.default_rng(0)
    D, V, k = 40, 800, 20
    c = random_corpus(rng, D, V, 1, 60, empty_every=9)
    lam = rng.gamma(100, 0.01, size=(V, k))
    eeb = oracle.topics_exp_elog_beta(lam)
    alpha = np.full(k, 1.0 / k)
    g0 = rng.gamma(100, 0.01, size=(D, k))
    g, its, _ = co.estep(c.indptr, c.indices, c.values, np.arange(D), eeb, alpha, g0, n_threads=4)
    for i in range(D):
        ids, cts = c.row(i)
        if ids.size == 0:
            assert np.all(g[i] == 0) and its[i] == 0
            continue
        go, _, it = oracle.variational_topic_inference(ids, cts, eeb, alpha, g0[i])
        assert it == its[i]
        np.testing.assert_allclose(g[i], go, rtol=1e-12)


def test_c_oracle_reference_books(co, oracle):
    """The C restatement also reproduces LDALoader.scala:108's recorded topic distributions."""
    tf = golden_npz("en_idf.npz")
    nwk = golden_npz("en_topics.npz")["nwk"]
    meta = golden_json("en_topicdist.json")
    eeb = oracle.topics_exp_elog_beta(nwk)
    g0 = np.stack([oracle.gamma_init(7, d, 5) for d in range(51)])
    g, _, _ = co.estep(tf["indptr"], tf["indices"], tf["tf"].astype(float), np.arange(51), eeb,
                       np.asarray(meta["docConcentration"]), g0)
    p = g / g.sum(axis=1, keepdims=True)
    exp = np.array([[float(x) for x in r] for r in meta["Result_EN_1591723228815"]])
    assert np.abs(p - exp).max() < 1e-6
