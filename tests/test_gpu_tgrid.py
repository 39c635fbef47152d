"""GPU: the fp64 many-topic team kernel with the topics split and the rows64 grid inside each member
(lda_team64.hip k_estep_tgrid64 — BASELINE config 4's k = 500 E-step), through the C ABI.

STC_TGRID=2 makes any fp64 many-topic launch that cannot take this kernel an error, so every call below
provably ran it.  Checked against the oracle's variationalTopicInference (γ ≤ 1e-7 with equal iteration
counts, a document on the stop rule's boundary compared to the same iteration; sstats 1e-10
mass-weighted), against the one-CU many-topic kernel over many uneven documents (teams finish documents
at different times, so the epoch granules are exercised across thousands of exchanges), through whole
training steps and topicDistribution, and with a member that never publishes (the call re-runs on the
one-CU kernel and returns results bit-identical to that kernel's)."""
import numpy as np
import pytest

from helpers import random_corpus

pytestmark = pytest.mark.gpu


def _rows_corpus(rng, V, sizes):
    import stc

    rows = []
    for n in sizes:
        if n == 0:
            rows.append((np.zeros(0, np.int32), np.zeros(0)))
            continue
        ids = np.sort(rng.choice(V, size=n, replace=False)).astype(np.int32)
        rows.append((ids, rng.integers(1, 7, ids.size).astype(np.float64)))
    return stc.CsrMatrix.from_rows(rows, V)


def _handle(ctx, corpus, k, lam, **kw):
    import stc

    h = stc.LdaHandle(ctx, k, corpus.num_cols, dtype="f64", **kw)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h.set_corpus(d, corpus.num_rows)
    h.set_topics(lam)
    return h, d


# row counts covering every row-set count R = 1..7 (64 rows per set), set boundaries, the cap, empty rows
SIZES = [1, 7, 63, 64, 65, 128, 129, 200, 256, 257, 320, 383, 384, 385, 400, 447, 448, 0, 372, 371, 12, 90]


@pytest.mark.parametrize("k", [105, 208, 300, 500, 700])
def test_tgrid_estep_vs_oracle(ctx, oracle, k, monkeypatch):
    monkeypatch.setenv("STC_TGRID", "2")
    rng = np.random.default_rng(400 + k)
    V = 4096
    corpus = _rows_corpus(rng, V, SIZES)
    D = corpus.num_rows
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    h, _ = _handle(ctx, corpus, k, lam)
    gamma, stat, iters = h.estep(np.arange(D), g0, want_stat=True)
    eeb = oracle.topics_exp_elog_beta(lam)
    alpha = np.full(k, 1.0 / k)
    stat_o = np.zeros((V, k))
    borderline = 0
    for i in range(D):
        cid, cts = corpus.row(i)
        if cid.size == 0:
            assert np.all(gamma[i] == 0) and iters[i] == 0
            continue
        g, ss, it = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i])
        if iters[i] != it:  # the stop rule's boundary (summation order decides): at most one document
            assert abs(int(iters[i]) - it) <= 1, (i, iters[i], it)
            borderline += 1
            assert borderline <= 1, (i, iters[i], it)
            g, ss, _ = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i], n_iter=int(iters[i]))
        np.testing.assert_allclose(gamma[i], g, rtol=1e-7)
        np.add.at(stat_o, cid, ss.T)
    nz = stat_o > 1e-8 * stat_o.max()
    assert (np.abs(stat[nz] - stat_o[nz]) / stat_o[nz]).max() < 1e-7
    assert np.abs(stat - stat_o).sum() / stat_o.sum() < 1e-10


def test_tgrid_many_documents_vs_the_one_cu_kernel(ctx, monkeypatch):
    """1500 documents of 300–448 rows at k = 500 (config 4's shape): γ and the iteration counts of the grid
    team against the one-CU many-topic kernel (STC_WIDE_TEAM=1) on the same inputs."""
    rng = np.random.default_rng(77)
    D, V, k = 1500, 8192, 500
    corpus = random_corpus(rng, D, V, 300, 448, empty_every=211)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    out = {}
    for knob, team in (("2", None), ("0", "1")):
        monkeypatch.setenv("STC_TGRID", knob)
        if team:
            monkeypatch.setenv("STC_WIDE_TEAM", team)
        h, d = _handle(ctx, corpus, k, lam)
        out[knob] = h.estep(np.arange(D), g0, want_stat=True)
        h.close()
        d.free()
    g2, s2, i2 = out["2"]
    g1, s1, i1 = out["0"]
    same = i2 == i1
    assert (~same).sum() <= 3, np.flatnonzero(~same)
    big = g1[same] >= 1.0
    np.testing.assert_allclose(g2[same][big], g1[same][big], rtol=1e-9)
    np.testing.assert_allclose(s2.sum(), s1.sum(), rtol=1e-9)


def test_tgrid_training_steps_and_topic_distribution_vs_oracle(ctx, oracle, monkeypatch):
    """Whole submitMiniBatch steps through the grid team (its eθ / E[log θ] / r / key outputs feed the
    sstats SpMM, logphat and the M-step) and topicDistribution (no sstats outputs), k = 500."""
    monkeypatch.setenv("STC_TGRID", "2")
    rng = np.random.default_rng(5)
    D, V, k = 120, 3000, 500
    corpus = random_corpus(rng, D, V, 1, 448, empty_every=29)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    h, d = _handle(ctx, corpus, k, lam0, mini_batch_fraction=0.4, optimize_doc_concentration=True)
    alpha, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D, mini_batch_fraction=0.4,
                               optimize_doc_concentration=True)
    for _ in range(2):
        ids = rng.integers(0, D, size=45)
        g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
        h.step(ids, g0)
        oracle.submit_minibatch(st, [corpus.row(i) for i in ids], list(g0))
    assert np.max(np.abs(h.topics() - st.lam.T) / st.lam.T) < 1e-9
    np.testing.assert_allclose(h.alpha(), st.alpha, rtol=1e-9)
    gd = rng.gamma(100.0, 0.01, size=(D, k))
    td = h.topic_distribution(d, gamma0=gd)
    for i in range(0, D, 7):
        cid, cts = corpus.row(i)
        want = oracle.topic_distribution(cid, cts, h.topics(), h.alpha(), gd[i])
        np.testing.assert_allclose(td[i], want, rtol=1e-7, atol=1e-12)


def test_tgrid_timeout_falls_back_to_the_one_cu_kernel(ctx, monkeypatch):
    """Member 1 of team 0 never publishes (STC_TEAM_FAULT=1): its partners give up, and the same call re-runs
    the launch on the one-CU kernel — λ, α and topicDistribution bit-identical to STC_TGRID=0 / one CU."""
    rng = np.random.default_rng(9)
    D, V, k = 48, 2048, 500
    corpus = random_corpus(rng, D, V, 100, 400)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    ids = np.arange(D)

    def run(knob, fault):
        monkeypatch.setenv("STC_TGRID", knob)
        if knob == "0":
            monkeypatch.setenv("STC_WIDE_TEAM", "1")
        else:
            monkeypatch.delenv("STC_WIDE_TEAM", raising=False)
        if fault:
            monkeypatch.setenv("STC_TEAM_FAULT", "1")
        else:
            monkeypatch.delenv("STC_TEAM_FAULT", raising=False)
        h, d = _handle(ctx, corpus, k, lam)
        h.step(ids, g0)
        td = h.topic_distribution(d, gamma0=g0)
        out = (h.topics(), h.alpha(), td)
        h.close()
        d.free()
        return out

    one = run("0", False)
    fb = run("2", True)
    for a, b in zip(fb, one):
        np.testing.assert_array_equal(a, b)
    healthy = run("2", False)
    np.testing.assert_allclose(healthy[0], one[0], rtol=1e-9)
