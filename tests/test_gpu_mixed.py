"""GPU: the mixed mode (STC_MIXED) — the fp32 E-step for every document, then the documents
whose fp32 fixed point took more than `mixed_resolve_iters` iterations re-solved in fp64 from the same γ₀
(api.hip mixed_resolve).

Checked against the two pure-precision handles on the same λ, documents and γ₀:
  * a re-solved document (fp32 iterations above the threshold) is the fp64 handle's: same iteration count,
    γ within fp32 storage rounding (the step buffers are fp32);
  * every other document is the fp32 handle's, bit for bit (the mixed handle's fp32 pass is the fp32 path);
  * the launch counters count exactly the documents above the threshold, through both re-solve lists (the
    fp64 fast kernel's documents and, past its row capacity, the workgroup kernel's).
The north-star bars (topicsMatrix 1e-4, logPerplexity 1e-5, identical top-10 terms) for this mode are in
tests/test_gpu_config1.py."""
import numpy as np
import pytest

from helpers import random_corpus

pytestmark = pytest.mark.gpu


def _handle(ctx, corpus, k, dtype, lam, **kw):
    import stc

    h = stc.LdaHandle(ctx, k, corpus.num_cols, dtype=dtype, **kw)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if dtype == "f32" else stc.STC_F64)
    h.set_corpus(d, corpus.num_rows)
    h.set_topics(lam)
    return h, d


@pytest.mark.parametrize("k", [40, 100])
def test_mixed_resolves_exactly_the_slow_documents(ctx, k):
    import stc

    rng = np.random.default_rng(600 + k)
    V = 3000
    short = random_corpus(rng, 1200, V, 10, 200, empty_every=37)
    longer = random_corpus(rng, 40, V, 260, 420)  # past the fp64 fast kernel's 256 rows: the long list
    rows = [short.row(i) for i in range(short.num_rows)] + [longer.row(i) for i in range(longer.num_rows)]
    corpus = stc.CsrMatrix.from_rows(rows, V)
    D = corpus.num_rows
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    ids = rng.permutation(D)
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    h64, _ = _handle(ctx, corpus, k, "f64", lam)
    h32, _ = _handle(ctx, corpus, k, "f32", lam)
    g64, _, it64 = h64.estep(ids, g0)
    g32, _, it32 = h32.estep(ids, g0)
    thr = int(np.percentile(it32[it32 > 0], 60))  # about 40 % of the documents above it
    hm, _ = _handle(ctx, corpus, k, "mixed", lam, mixed_resolve_iters=thr)
    c0 = hm.counters()["kernels"]
    gm, _, itm = hm.estep(ids, g0)
    c1 = hm.counters()["kernels"]
    slow = it32 > thr
    nnz = np.diff(corpus.indptr)[ids]
    assert slow.sum() > 50 and (slow & (nnz > 256)).sum() > 3 and (~slow & (it32 > 0)).sum() > 50
    assert c1["mixed_docs"] - c0["mixed_docs"] == slow.sum()
    assert c1["mixed_resolves"] - c0["mixed_resolves"] == 1
    np.testing.assert_array_equal(itm[slow], it64[slow])
    np.testing.assert_allclose(gm[slow], g64[slow], rtol=2e-7, atol=1e-30)
    np.testing.assert_array_equal(itm[~slow], it32[~slow])
    np.testing.assert_array_equal(gm[~slow], g32[~slow])


def test_mixed_training_steps_and_inference(ctx, oracle):
    """Injected λ₀ / membership / γ₀ through mixed training steps (the low threshold re-solves a share of
    each batch): λ / α against the oracle, the bound and topicDistribution of a mixed handle in fp64 (its
    inference path) equal to the fp64 handle's on the same λ."""
    import stc

    rng = np.random.default_rng(61)
    D, V, k = 300, 2000, 24
    corpus = random_corpus(rng, D, V, 1, 120, empty_every=19)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    hm, dm = _handle(ctx, corpus, k, "mixed", lam0, mini_batch_fraction=0.3, optimize_doc_concentration=True,
                     mixed_resolve_iters=300)
    alpha, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D, mini_batch_fraction=0.3,
                               optimize_doc_concentration=True)
    c0 = hm.counters()["kernels"]
    for _ in range(3):
        ids = np.sort(rng.choice(D, size=100, replace=True))
        g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
        hm.step(ids, g0)
        oracle.submit_minibatch(st, [corpus.row(i) for i in ids], list(g0))
    assert hm.counters()["kernels"]["mixed_docs"] > c0["mixed_docs"]
    lam = hm.topics()
    assert np.max(np.abs(lam - st.lam.T) / st.lam.T) < 1e-4
    np.testing.assert_allclose(hm.alpha(), st.alpha, rtol=1e-4)
    # inference in fp64 on the mixed handle's λ
    h64, d64 = _handle(ctx, corpus, k, "f64", lam)
    h64.set_alpha(hm.alpha())
    bm, b64 = hm.bound(dm, gamma_seed=5), h64.bound(d64, gamma_seed=5)
    np.testing.assert_allclose(bm["bound"], b64["bound"], rtol=1e-12)
    np.testing.assert_allclose(hm.topic_distribution(dm, gamma_seed=5), h64.topic_distribution(d64, gamma_seed=5),
                               rtol=1e-12, atol=1e-15)


def test_mixed_next_and_group(ctx):
    """Device-sampled next() through a mixed handle and a mixed two-member group (in-process transport, the
    fp64 rows all-gathered beside the fp32 ones): both train (finite λ, iterations counted) and both re-solve
    documents in fp64."""
    import stc

    rng = np.random.default_rng(62)
    D, V, k = 600, 2500, 30
    corpus = random_corpus(rng, D, V, 5, 150, empty_every=23)
    kw = dict(mini_batch_fraction=0.2, seed=9, optimize_doc_concentration=True, dtype="mixed", mixed_resolve_iters=50)
    h = stc.LdaHandle(ctx, k, V, **kw)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h.set_corpus(d, D)
    h.init_random(3)
    for _ in range(4):
        h.next()
    with stc.LdaGroup([0, 0], k, V, **kw) as g:
        g.set_corpus(corpus)
        g.init_random(3)
        for _ in range(4):
            g.next()
        assert g.iteration() == h.iteration() == 4
        assert np.all(np.isfinite(g.topics()))
        assert sum(c["kernels"]["mixed_docs"] for c in g.counters()) > 0
    assert h.counters()["kernels"]["mixed_docs"] > 0
