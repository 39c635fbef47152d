"""BASELINE configs[0] end to end — the reference's own flow (LDAClustering.scala:23-61): term
frequencies → IDF(minDocFreq = 2) with the 1e-4 floor (:177-188) → online LDA, k = 20, 10 iterations,
miniBatchFraction = 0.05 + 1/N (:43), optimizeDocConcentration false (mllib OnlineLDAOptimizer's
default), α = η = 1/k (Params.scala:1-11: −1 ⇒ auto).

20 Newsgroups is not in the container; the stand-in is the reference's own EN corpus: 51 books whose
per-document term counts are recovered exactly from the saved model (fixture F1, en_idf.npz) and whose
term strings are that model's vocabulary (F5, en_vocab.txt).  Each book becomes its token stream (term
i repeated tf times, 2.1M tokens) and goes through HashingTF (2^18 buckets, Spark 2.4.3's murmur3
tail) on the GPU, so the TF vectors are the north star's hashed ones.

Spark's MT19937 draws (λ₀, minibatch membership, γ₀) cannot be replayed without a JVM, so they are
injected — identical inputs on both sides — and the GPU's 10 stc_lda_step calls are compared with
the oracle's 10 submit_minibatch calls against the north-star bars (topicsMatrix within 1e-4
relative, logPerplexity within 1e-5 relative, identical top-10 terms per topic): the fp64 path (Spark's
precision) at 1e-9 / 1e-10 with identical top-10 terms; the mixed mode (STC_MIXED: the fp32 E-step, the
documents past 500 fp32 iterations re-solved in fp64) at the north-star bars themselves, 1e-4 / 1e-5 with
identical top-10 terms; the fp32 path at 1e-3 on the topicsMatrix (see below), 1e-5 on logPerplexity,
identical top-10 terms.
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, golden_npz

pytestmark = pytest.mark.gpu

K, ITERS, NF = 20, 10, 1 << 18


@pytest.fixture(scope="module")
def books():
    tf = golden_npz("en_idf.npz")
    vocab = open(os.path.join(GOLDEN, "en_vocab.txt"), encoding="utf-8").read().split("\n")[:-1]
    assert len(vocab) == int(tf["vocab_size"])
    ip, ix, cnt = tf["indptr"], tf["indices"], tf["tf"]
    docs = [[vocab[i] for i, c in zip(ix[ip[d]:ip[d + 1]], cnt[ip[d]:ip[d + 1]]) for _ in range(int(c))]
            for d in range(ip.size - 1)]
    return tf, vocab, docs


def _oracle_tf(oracle, tf, vocab):
    """HashingTF of the books from the vocabulary's buckets (the same counts, aggregated per bucket)."""
    bucket = np.array([oracle.non_negative_mod(oracle.murmur3_x86_32(w.encode("utf-8"), 42, oracle.HASH_SPARK24), NF)
                       for w in vocab], np.int64)
    ip, ix, cnt = tf["indptr"], tf["indices"], tf["tf"]
    indptr, idx, val = [0], [], []
    for d in range(ip.size - 1):
        b = bucket[ix[ip[d]:ip[d + 1]]]
        u, inv = np.unique(b, return_inverse=True)
        c = np.zeros(u.size)
        np.add.at(c, inv, cnt[ip[d]:ip[d + 1]].astype(np.float64))
        idx.append(u.astype(np.int32))
        val.append(c)
        indptr.append(indptr[-1] + u.size)
    return np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(val)


def test_config1_pipeline_hashing_idf_online_lda(ctx, oracle, books):
    import stc

    tf, vocab, docs = books
    D = len(docs)
    # ---- HashingTF (GPU) vs the oracle: bit-exact indices and counts
    d_tf = stc.HashingTF(numFeatures=NF, ctx=ctx).transform_device(docs)
    got = d_tf.download()
    ip_o, ix_o, vv_o = _oracle_tf(oracle, tf, vocab)
    assert np.array_equal(got.indptr, ip_o) and np.array_equal(got.indices, ix_o) and np.array_equal(got.values, vv_o)
    assert got.values.sum() == tf["tf"].sum()
    # ---- IDF(2) + the reference's 1e-4 floor (GPU, in place on the device CSR)
    model = stc.IDF(minDocFreq=2, ctx=ctx).fit_device(d_tf)
    idf_o, df_o, m_o = oracle.idf_fit(ip_o, ix_o, vv_o, NF, 2)
    assert model.numDocs == m_o == D and np.array_equal(model.docFreq, df_o)
    np.testing.assert_allclose(model.idf, idf_o, rtol=1e-15, atol=0)
    model.transform_device(d_tf, zero_floor=1e-4)
    corpus = d_tf.download()
    np.testing.assert_allclose(corpus.values, oracle.idf_transform(ix_o, vv_o, idf_o, floor=1e-4), rtol=1e-15, atol=0)
    d_tf.free()

    # ---- online LDA, k = 20, 10 iterations, injected λ₀ / membership / γ₀
    rng = np.random.default_rng(2020)
    frac = stc.reference_mini_batch_fraction(D)
    lam0 = rng.gamma(100.0, 0.01, size=(NF, K))
    batches = []
    for _ in range(ITERS):
        ids = np.flatnonzero(rng.random(D) < frac)
        if ids.size == 0:  # Spark would skip the step without an iteration; keep ten real steps
            ids = rng.choice(D, size=1)
        batches.append((ids, rng.gamma(100.0, 0.01, size=(ids.size, K))))
    g_bound = rng.gamma(100.0, 0.01, size=(D, K))
    alpha, eta = oracle.resolve_alpha_eta(K)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D, mini_batch_fraction=frac,
                               optimize_doc_concentration=False)
    rows = [corpus.row(i) for i in range(D)]
    for ids, g0 in batches:
        oracle.submit_minibatch(st, [rows[i] for i in ids], list(g0))
    lp_o = oracle.log_perplexity(rows, list(g_bound), st.lam.T, st.alpha, eta)
    idx_o, _ = oracle.describe_topics(st.lam.T, 10)

    # fp32: the first minibatch holds a book whose E-step takes ≈3300 iterations from the random λ₀; Spark's
    # stopping rule (mean |Δγ| ≤ 1e-3) leaves that slowly contracting fixed point O(1e-3)·γ short of
    # convergence, and the fp32 trajectory stops at a different iterate than the fp64 one: measured
    # 4.8e-4 relative on the topicsMatrix, so fp32 gets 1e-3 here (the fp64 path meets the north-star
    # 1e-4 bar by five orders of magnitude)
    # mixed: that book (and the two at ≈ 575 iterations) are re-solved in fp64, every other document keeps its
    # fp32 E-step — the north-star bars hold (tools: the CPU emulation in DESIGN.md §4 predicts ≈ 2e-7)
    for dtype, tol_lam, tol_lp in (("f64", 1e-9, 1e-10), ("mixed", 1e-4, 1e-5), ("f32", 1e-3, 1e-5)):
        h = stc.LdaHandle(ctx, K, NF, mini_batch_fraction=frac, optimize_doc_concentration=False, dtype=dtype)
        dc = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if dtype == "f32" else stc.STC_F64)
        h.set_corpus(dc, D)
        h.set_topics(lam0)
        for ids, g0 in batches:
            h.step(ids, g0)
        assert h.iteration() == ITERS
        lam = h.topics()
        rel = np.max(np.abs(lam - st.lam.T) / st.lam.T)
        assert rel < tol_lam, (dtype, rel)
        lda_model = stc.LDAModel(h)
        lp = lda_model.logPerplexity(dc, gamma0=g_bound)
        assert abs(lp - lp_o) / abs(lp_o) < tol_lp, (dtype, lp, lp_o)
        idx, _ = h.describe(10)
        assert np.array_equal(idx, idx_o), dtype
        if dtype == "mixed":  # the slow books went through the fp64 re-solve
            assert h.counters()["kernels"]["mixed_docs"] >= 3
        print(f"config1 {dtype}: topicsMatrix rel {rel:.3e}, logPerplexity rel {abs(lp - lp_o) / abs(lp_o):.3e}")
        dc.free()
