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


@pytest.mark.parametrize("optimize_alpha", [True, False])
def test_c_oracle_minibatch_matches_numpy_oracle(co, oracle, optimize_alpha):
    """oracle_minibatch (the bench's full-step CPU baseline) = submit_minibatch of the NumPy oracle."""
    rng = np.random.default_rng(1)
    D, V, k = 60, 500, 8
    c = random_corpus(rng, D, V, 1, 40, empty_every=7)
    lam0 = rng.gamma(100, 0.01, size=(V, k))
    ids = np.sort(rng.choice(D, size=25, replace=True))
    g0 = rng.gamma(100, 0.01, size=(ids.size, k))
    alpha, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha.copy(), eta=eta, corpus_size=D,
                               mini_batch_fraction=0.4, optimize_doc_concentration=optimize_alpha)
    st.iteration = 4
    oracle.submit_minibatch(st, [c.row(i) for i in ids], list(g0))
    lam = np.ascontiguousarray(lam0.T)
    a = alpha.copy()
    rho = (1024.0 + 5) ** -0.51
    scale = D / np.ceil(0.4 * D)
    tot = co.minibatch(c.indptr, c.indices, c.values, ids, g0, lam, a, eta, rho, scale, optimize_alpha,
                       n_threads=4)
    assert tot > 0
    np.testing.assert_allclose(lam, st.lam, rtol=1e-12)
    np.testing.assert_allclose(a, st.alpha, rtol=1e-12)
