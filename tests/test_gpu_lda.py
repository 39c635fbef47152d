"""GPU parity for the online-LDA path (K6–K12) through the C ABI vs the CPU oracle and the
reference's known answers (tests/golden/en_topicdist.json, en_describe.json).

Tolerances: f64 mode (the default and the benchmark headline) restates Spark's double arithmetic, so
λ/γ/bound agree to ~1e-9 relative and meets the north-star bars (topicsMatrix 1e-4, logPerplexity 1e-5,
identical top-10 terms) everywhere.  f32 mode (the fast secondary) is held to those bars on the synthetic
cases here, but it does NOT meet the topicsMatrix bar on configs[0]: one book's E-step takes ≈3300
iterations there and the fp32 trajectory stops at another iterate (4.8e-4 relative,
test_gpu_config1.py), so fp32 is not a north-star-parity mode and every fp32 bench line says so.
"""
import numpy as np
import pytest

from helpers import golden_json, golden_npz, long_run_corpus, planted_corpus, random_corpus

pytestmark = pytest.mark.gpu

TOL = {"f64": dict(lam=1e-9, gamma=1e-7, bound=1e-10), "f32": dict(lam=1e-4, gamma=2e-3, bound=1e-5)}


def _handle(ctx, corpus, k, dtype, lam=None, **kw):
    import stc

    h = stc.LdaHandle(ctx, k, corpus.num_cols, dtype=dtype, **kw)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if dtype == "f32" else stc.STC_F64)
    h.set_corpus(d, kw.pop("corpus_total", corpus.num_rows))
    if lam is not None:
        h.set_topics(lam)
    return h, d


@pytest.mark.parametrize("dtype,k,kernel", [("f64", 16, "wg"), ("f32", 16, "wave"), ("f32", 16, "wg"),
                                             ("f32", 100, "wave"), ("f32", 100, "wg"), ("f32", 128, "wave"),
                                             ("f32", 77, "wave"), ("f64", 100, "wave"), ("f64", 100, "wg"),
                                             ("f64", 40, "wave"), ("f64", 20, "wave"), ("f64", 104, "wave"),
                                             ("f32", 300, "wave"), ("f64", 300, "wave"), ("f32", 700, "wave"),
                                             ("f64", 700, "wave"), ("f32", 1500, "wave"), ("f64", 1500, "wave"),
                                             ("f64", 300, "team1"), ("f64", 300, "team2"), ("f64", 700, "team3"),
                                             ("f32", 700, "team2"), ("f64", 1500, "team4")])
def test_estep_gamma_and_stat(ctx, oracle, dtype, k, kernel, monkeypatch):
    """Every E-step kernel vs the oracle: the register-resident grid kernels (fp32 k <= 128, fp64
    k <= 104 with R = 1..6 row sets, the sixth from LDS), the many-topic kernel (k > 128 / 104: Q = 1, 2,
    4 topics per lane; rows in VGPRs, then LDS, then streamed from global memory — docs up to 600 terms
    reach all three), the same with each document's rows split over a team of P = 1..4 CUs
    (k_estep_wide_mc, "teamP") and the workgroup-per-doc kernel (docs past the fast kernels' row
    capacity)."""
    if kernel == "wg":
        monkeypatch.setenv("STC_DISABLE_WAVE", "1")
    if kernel.startswith("team"):  # many-topic kernel with a forced team of P CUs per document
        monkeypatch.setenv("STC_WIDE_TEAM", kernel[4:])
    rng = np.random.default_rng(10 + k)
    D, V = 48, 2048
    corpus = random_corpus(rng, D, V, 1, 600 if k > 128 else 300, empty_every=13)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    h, _ = _handle(ctx, corpus, k, dtype, lam)
    ids = np.arange(D)
    gamma, stat, iters = h.estep(ids, g0, want_stat=True)
    eeb = oracle.topics_exp_elog_beta(lam)
    alpha = np.full(k, 1.0 / k)
    stat_o = np.zeros((V, k))
    borderline = 0
    for i in ids:
        cid, cts = corpus.row(i)
        if cid.size == 0:
            assert np.all(gamma[i] == 0) and iters[i] == 0
            continue
        g, ss, it = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i])
        if iters[i] != it:
            # Spark's stop rule mean |Δγ| ≤ 1e-3 lets the last iteration move Σ|γ| by up to 1e-3·k (1.5 at
            # k = 1500), so a run that stops an iteration apart lands visibly elsewhere: in fp64 only when
            # the test sat on the boundary (summation order decides, at most one doc), in fp32 when
            # rounding moves the crossing.  Both are compared with the oracle run to the same iteration.
            assert abs(int(iters[i]) - it) <= (1 if dtype == "f64" else 3), (i, iters[i], it)
            if dtype == "f64":
                borderline += 1
                assert borderline <= 1, (i, iters[i], it)
            g, ss, _ = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i], n_iter=int(iters[i]))
        if dtype == "f64":
            np.testing.assert_allclose(gamma[i], g, rtol=TOL[dtype]["gamma"])
        else:  # fp32 vs fp64 at the same iteration: rounding proportional to the doc's mass on the whole
            # vector, 2e-3 relative on topics holding ≥ 1 token's mass
            l1 = np.abs(gamma[i] - g).sum()
            assert l1 <= 1e-3 * k + 1e-4 * g.sum(), (i, l1, g.sum())
            big = g >= 1.0
            np.testing.assert_allclose(gamma[i][big], g[big], rtol=TOL[dtype]["gamma"])
        np.add.at(stat_o, cid, ss.T)
    # fp32: a topic dying towards α (γ ~ 1e-3) has eθ ∝ exp(ψ(γ)) with dψ = dγ/γ², so its few sstats
    # entries carry fp32's γ rounding ×1e6 (at γ ~ 0.02, ×2500) — mass-weighted error 1e-4 over all
    # entries, and relative 1e-2 on entries ≥ 1e-4 of the largest
    nz = stat_o > (1e-8 if dtype == "f64" else 1e-4) * stat_o.max()
    rel = np.abs(stat[nz] - stat_o[nz]) / stat_o[nz]
    if dtype == "f64":  # the same amplification at fp64 rounding: γ's 1e-7 bound, 1e-10 mass-weighted
        assert rel.max() < TOL[dtype]["gamma"], rel.max()
        assert np.abs(stat - stat_o).sum() / stat_o.sum() < 1e-10
        assert np.all(stat[~nz] < 1e-6 * stat_o.max() + 1e-300)
    else:
        l1 = np.abs(stat - stat_o).sum() / stat_o.sum()
        assert l1 < 1e-4, l1
        assert rel.max() < 1e-2, rel.max()


@pytest.mark.parametrize("k,scale", [(100, 5e4), (100, 5e5), (300, 5e5)])
def test_estep_fp32_at_production_scale_lambda(ctx, oracle, k, scale):
    """the fp32 E-step carries expElogβ's per-topic factor exp(−ψ(colsum_t)) in eθ', so a λ of
    a large corpus (colsum 1e8–1e9 here: λ scaled by 5e4–5e5 over V = 2048) scales eθ' and φ down by
    that much.  γ still matches the fp64 oracle within the fp32 bounds of test_estep_gamma_and_stat."""
    rng = np.random.default_rng(70 + k)
    D, V = 40, 2048
    corpus = random_corpus(rng, D, V, 1, 300, empty_every=11)
    lam = rng.gamma(100.0, 0.01, size=(V, k)) * scale * rng.uniform(0.5, 2.0, size=(V, 1))
    assert lam.sum(axis=0).min() > 1e8 * (scale / 5e5)
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    h, _ = _handle(ctx, corpus, k, "f32", lam)
    gamma, _, iters = h.estep(np.arange(D), g0)
    eeb = oracle.topics_exp_elog_beta(lam)
    alpha = np.full(k, 1.0 / k)
    for i in range(D):
        cid, cts = corpus.row(i)
        if cid.size == 0:
            continue
        g, _, it = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i])
        assert abs(int(iters[i]) - it) <= 3, (i, iters[i], it)
        if iters[i] != it:
            g, _, _ = oracle.variational_topic_inference(cid, cts, eeb, alpha, g0[i], n_iter=int(iters[i]))
        assert np.abs(gamma[i] - g).sum() <= 1e-3 * k + 1e-4 * g.sum(), (i, np.abs(gamma[i] - g).sum())
        big = g >= 1.0
        np.testing.assert_allclose(gamma[i][big], g[big], rtol=TOL["f32"]["gamma"])


@pytest.mark.parametrize("dtype,k", [("f64", 16), ("f64", 100), ("f64", 300), ("f32", 100), ("f32", 700)])
def test_sstats_long_runs_over_tiles(ctx, oracle, dtype, k):
    """sstats where frequent terms' runs span hundreds of chunks (k_fixup walks full tiles): stat vs
    Spark's sstats rebuilt on the host from the kernel's own γ (eθ = exp(ψ(γ) − ψ(Σγ)) with Breeze's ψ,
    φnorm = eθ·expElogβ[:, ids] + 1e-100, stat[v] = Σ_d eθ_d · cnt_dv / φnorm_dv) — the summation of the
    run partials is all this checks, so the E-step's iterate is taken as given — and bitwise equal over
    two launches.  f64 1e-10 relative; f32 2e-3 per entry (fp32 ψ of a dying topic's γ ~ 1e-3 is off by
    ~6e-5 absolute, so its eθ by that relative) and 2e-4 on the hot rows (fp32 sums of ~2e4 entries)."""
    import scipy.sparse as sp

    rng = np.random.default_rng(5 + k)
    D, V = 24000, 4096
    corpus = long_run_corpus(rng, D, V, [0, 1, 2, 900, 901, 2047, 4095])
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    h, _ = _handle(ctx, corpus, k, dtype, lam)
    ids = np.arange(D)
    gamma, stat, _ = h.estep(ids, g0, want_stat=True)
    _, stat2, _ = h.estep(ids, g0, want_stat=True)
    np.testing.assert_array_equal(stat, stat2)
    eth = np.exp(oracle.dirichlet_expectation(gamma))  # D × k
    eeb = oracle.topics_exp_elog_beta(lam)  # V × k
    rows = np.repeat(np.arange(D), np.diff(corpus.indptr))
    phinorm = np.empty(corpus.indices.size)
    for s in range(0, rows.size, 1 << 14):  # bounded host memory at k = 700
        e = slice(s, s + (1 << 14))
        phinorm[e] = np.einsum("ij,ij->i", eth[rows[e]], eeb[corpus.indices[e]]) + 1e-100
    w = sp.csr_matrix((corpus.values / phinorm, (corpus.indices, rows)), shape=(V, D))
    ref = np.asarray(w @ eth)
    assert np.count_nonzero(corpus.indices == 0) == D  # term 0's run: D entries, D / 256 chunks
    big = ref > 1e-6 * ref.max()
    rel = np.abs(stat[big] - ref[big]) / ref[big]
    assert rel.max() < (1e-10 if dtype == "f64" else 2e-3), rel.max()
    hot = [0, 1, 2, 900, 901, 2047, 4095]  # the long runs: a lost or doubled tile is percent-level here
    np.testing.assert_allclose(stat[hot], ref[hot], rtol=1e-10 if dtype == "f64" else 2e-4,
                               atol=1e-6 * ref.max())  # fp32 flushes entries ~1e-37 to zero


def test_estep_long_documents_global_path(ctx, oracle):
    """Docs whose nnz×k block exceeds the LDS budget stream it from L2 instead (books-sized rows)."""
    rng = np.random.default_rng(11)
    D, V, k = 6, 20000, 5
    corpus = random_corpus(rng, D, V, 3000, 12000, max_count=40)
    lam = rng.gamma(100.0, 0.01, size=(V, k)) * rng.uniform(0.1, 10.0, size=(V, 1))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    for dtype in ("f64", "f32"):
        h, _ = _handle(ctx, corpus, k, dtype, lam)
        gamma, _, _ = h.estep(np.arange(D), g0)
        eeb = oracle.topics_exp_elog_beta(lam)
        for i in range(D):
            cid, cts = corpus.row(i)
            g, _, _ = oracle.variational_topic_inference(cid, cts, eeb, np.full(k, 1.0 / k), g0[i])
            np.testing.assert_allclose(gamma[i], g, rtol=TOL[dtype]["gamma"])


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("optimize_alpha,k", [(True, 12), (False, 12), (True, 300)])
def test_minibatch_steps_match_oracle(ctx, oracle, dtype, optimize_alpha, k):
    """Injected λ₀, membership (with duplicates) and γ₀: λ and α after 3 submitMiniBatch calls (k = 300:
    the many-topic E-step and the row-per-workgroup M-step pass)."""
    rng = np.random.default_rng(12)
    D, V = 80, 1024
    corpus = random_corpus(rng, D, V, 1, 60, empty_every=17)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    frac = 0.3
    h, _ = _handle(ctx, corpus, k, dtype, lam0, mini_batch_fraction=frac,
                   optimize_doc_concentration=optimize_alpha)
    alpha, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D,
                               mini_batch_fraction=frac, optimize_doc_concentration=optimize_alpha)
    for it in range(3):
        ids = np.sort(rng.choice(D, size=30, replace=True))
        g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
        s = h.step(ids, g0)
        oracle.submit_minibatch(st, [corpus.row(i) for i in ids], list(g0))
        assert s["batch_docs"] == ids.size
        assert s["nonempty_docs"] == sum(corpus.row(i)[0].size > 0 for i in ids)
        assert abs(s["rho"] - st.rho()) < 1e-15
    assert h.iteration() == 3
    lam = h.topics()
    rel = np.max(np.abs(lam - st.lam.T) / st.lam.T)
    assert rel < TOL[dtype]["lam"], rel
    np.testing.assert_allclose(h.alpha(), st.alpha, rtol=TOL[dtype]["lam"])
    # identical top-10 terms per topic
    idx, w = h.describe(10)
    idx_o, w_o = oracle.describe_topics(st.lam.T, 10)
    if dtype == "f64":
        assert np.array_equal(idx, idx_o)
    np.testing.assert_allclose(np.sort(w, axis=1), np.sort(w_o, axis=1), rtol=TOL[dtype]["lam"])


def test_all_empty_batch_is_a_no_op(ctx, oracle):
    rng = np.random.default_rng(13)
    V, k = 256, 4
    import stc

    corpus = stc.CsrMatrix.from_rows([(np.zeros(0, np.int32), np.zeros(0))] * 5, V)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    h, _ = _handle(ctx, corpus, k, "f64", lam0)
    s = h.step(np.arange(5))
    assert s["nonempty_docs"] == 0
    assert h.iteration() == 1  # Spark: iteration += 1 happens before the empty check
    np.testing.assert_array_equal(h.topics(), lam0)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_log_likelihood_and_perplexity(ctx, oracle, dtype):
    import stc

    rng = np.random.default_rng(14)
    D, V, k = 40, 1500, 8
    corpus, _ = planted_corpus(rng, D, V, k, L=50)
    lam = rng.gamma(100.0, 0.01, size=(V, k)) + rng.uniform(0, 50, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    alpha = rng.uniform(0.05, 0.5, size=k)
    model = stc.LDAModel.from_topics(lam, alpha, 0.07, dtype=dtype, ctx=ctx)
    ll = model.logLikelihood(corpus, gamma0=g0)
    lp = model.logPerplexity(corpus, gamma0=g0)
    docs = [corpus.row(i) for i in range(D)]
    b_o, cp_o, tp_o = oracle.log_likelihood_bound(docs, list(g0), lam, alpha, 0.07)
    lp_o = oracle.log_perplexity(docs, list(g0), lam, alpha, 0.07)
    assert abs(ll - b_o) / abs(b_o) < TOL[dtype]["bound"], (ll, b_o)
    assert abs(lp - lp_o) / abs(lp_o) < TOL[dtype]["bound"], (lp, lp_o)
    # the two parts separately (the topics part is pinned independently in test_bound_restatement.py)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if dtype == "f32" else stc.STC_F64)
    parts = model._h.bound(d, model.gammaSeed, 0, g0)
    assert abs(parts["corpus_part"] - cp_o) / abs(cp_o) < TOL[dtype]["bound"], (parts, cp_o)
    assert abs(parts["topics_part"] - tp_o) / abs(tp_o) < 1e-10, (parts, tp_o)  # fp64 on every path
    assert parts["token_count"] == sum(float(np.sum(c)) for _, c in docs)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_topic_distribution_reference_books(ctx, oracle, dtype):
    """LDALoader.scala:108 — the reference's 51 books × 5 topic proportions (two recorded Spark runs
    whose own spread is 7.1e-7) reproduced from the saved EM model's topicsMatrix with α = 11."""
    import stc

    tf = golden_npz("en_idf.npz")
    topics = golden_npz("en_topics.npz")["nwk"]
    meta = golden_json("en_topicdist.json")
    V = int(tf["vocab_size"])
    corpus = stc.CsrMatrix(tf["indptr"], tf["indices"], tf["tf"].astype(np.float64), V)
    model = stc.LDAModel.from_topics(topics, meta["docConcentration"], meta["topicConcentration"],
                                     gamma_shape=meta["gammaShape"], seed=7, dtype=dtype, ctx=ctx)
    got = model.transform(corpus)
    tol = 2e-6 if dtype == "f64" else 1e-5
    for run in ("Result_EN_1591066624209", "Result_EN_1591723228815"):
        exp = np.array([[float(x) for x in r] for r in meta[run]])
        err = np.abs(got - exp).max()
        assert err < tol, (run, err)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_describe_topics_reference(ctx, dtype):
    """Top terms + weights printed by the reference (Result_EN_*), from the saved topicsMatrix."""
    import stc

    topics = golden_npz("en_topics.npz")["nwk"]
    meta = golden_json("en_describe.json")
    model = stc.LDAModel.from_topics(topics, meta["docConcentration"], meta["topicConcentration"],
                                     dtype=dtype, ctx=ctx)
    desc = model.describeTopics(10)
    for run, tops in meta["describe"].items():
        for t, lst in tops.items():
            _, idx, w = desc[int(t)]
            for j, e in enumerate(lst):
                assert idx[j] == e["index"], (run, t, j)
                assert abs(w[j] - float(e["weight"])) / float(e["weight"]) < 1e-12


def test_next_device_sampling(ctx):
    """stc_lda_next: Poisson(f) membership per doc on the device; statistics of the batch sizes."""
    rng = np.random.default_rng(15)
    D, V, k = 4000, 4096, 10
    corpus = random_corpus(rng, D, V, 1, 30)
    h, _ = _handle(ctx, corpus, k, "f32", None, mini_batch_fraction=0.1, seed=5)
    h.init_random(5)
    sizes = []
    for _ in range(8):
        s = h.next()
        sizes.append(s["batch_docs"])
        assert s["cap_hits"] == 0 and s["inner_iters"] > 0
    assert abs(np.mean(sizes) - 400) < 4 * np.sqrt(400 / 8) + 10
    c = h.counters()
    assert c["docs"] == sum(sizes)
    assert np.all(np.isfinite(h.topics()))


def test_fit_pipeline_end_to_end(ctx, oracle):
    """HashingTF → IDF → LDA.fit(online) → describeTopics/logPerplexity/transform on a planted corpus;
    perplexity must drop below that of the initial random model."""
    import stc

    rng = np.random.default_rng(16)
    D, V, k = 600, 2000, 5
    corpus, _ = planted_corpus(rng, D, V, k, L=80, alpha=0.05)
    lda = stc.LDA(k=k, maxIter=30, subsamplingRate=0.2, seed=3, ctx=ctx)
    model = lda.fit(corpus)
    lp = model.logPerplexity(corpus)
    init = stc.LDA(k=k, maxIter=0, seed=3, ctx=ctx).fit(corpus)
    lp0 = init.logPerplexity(corpus)
    assert lp < lp0 - 0.2, (lp, lp0)
    theta = model.transform(corpus)
    np.testing.assert_allclose(theta.sum(axis=1), 1.0, rtol=1e-5)
    assert len(model.describeTopics(5)) == k


def test_model_save_load_round_trip_on_gpu(ctx, tmp_path):
    """LocalLDAModel.save → LocalLDAModel.load (Spark's directory layout) keeps the model exactly:
    same topicsMatrix, describeTopics and topicDistribution from the GPU."""
    import stc

    rng = np.random.default_rng(17)
    V, k, D = 700, 6, 20
    lam = rng.gamma(100.0, 0.01, size=(V, k)) * rng.uniform(0.5, 5.0, size=(V, 1))
    m = stc.LDAModel.from_topics(lam, rng.uniform(0.1, 0.5, size=k), 0.2, dtype="f64", ctx=ctx)
    path = str(tmp_path / "lda")
    m.save(path)
    m2 = stc.LDAModel.load(path, dtype="f64", ctx=ctx)
    assert np.array_equal(m2.topicsMatrix(), lam)
    assert np.array_equal(m2.estimatedDocConcentration(), m.estimatedDocConcentration())
    for (t1, i1, w1), (t2, i2, w2) in zip(m.describeTopics(8), m2.describeTopics(8)):
        assert t1 == t2 and np.array_equal(i1, i2) and np.array_equal(w1, w2)
    corpus = random_corpus(rng, D, V, 1, 40)
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    assert np.array_equal(m.transform(corpus, gamma0=g0), m2.transform(corpus, gamma0=g0))


def test_distributed_model_load_to_local_on_gpu(ctx, oracle, tmp_path):
    """The reference's flow (LDALoader.scala:37, :66, :108) on a synthetic EM model saved in the
    DistributedLDAModel layout: load → describeTopics → toLocal.topicDistribution, vs the oracle."""
    import stc

    rng = np.random.default_rng(18)
    V, k, D = 500, 5, 12
    nwk = rng.gamma(0.3, 20.0, size=(V, k))
    docs = random_corpus(rng, D, V, 5, 60)
    src = np.repeat(np.arange(D), np.diff(docs.indptr))
    stc.io.save_distributed(str(tmp_path / "em"), np.arange(D), rng.uniform(1, 9, size=(D, k)), nwk,
                            (src, docs.indices, docs.values), 11.0, 1.1)
    dm = stc.DistributedLDAModel.load(str(tmp_path / "em"))
    assert np.array_equal(dm.topicsMatrix(), nwk)
    idx_o, w_o = oracle.describe_topics(nwk, 10)
    for t, idx, w in dm.describeTopics(10, ctx=ctx):
        assert np.array_equal(idx, idx_o[t])
        np.testing.assert_allclose(w, w_o[t], rtol=1e-12)
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    theta = dm.toLocal(ctx=ctx).transform(docs, gamma0=g0)
    eeb = oracle.topics_exp_elog_beta(nwk)
    for i in range(D):
        cid, cts = docs.row(i)
        exp_t = oracle.topic_distribution(cid, cts, nwk, np.full(k, 11.0), g0[i], eeb)
        np.testing.assert_allclose(theta[i], exp_t, rtol=1e-7, atol=1e-12)


def _train(ctx, corpus, k, dtype, steps, reset_each=False, **kw):
    h, d = _handle(ctx, corpus, k, dtype, None, mini_batch_fraction=0.3, seed=9, **kw)
    h.init_random(4)
    for _ in range(steps):
        if reset_each:  # set_corpus drops the prefetched draw: every step samples synchronously
            h.set_corpus(d, corpus.num_rows)
        h.next(stats=False)
    return h, d


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("V,shards,k", [(1000, 3, 12), (100, 4, 12), (4096, 2, 12), (1000, 3, 300)])
def test_sharded_mstep_slices_bit_identical(ctx, monkeypatch, dtype, V, shards, k):
    """The multi-GPU M-step's vocabulary slices (ranks' λ / expElogβ rows, colsum partials placed
    where the one-GPU reduction has them), run on one GPU with STC_VIRTUAL_SHARDS: λ, α, the bound
    and topicDistribution are bit-identical to the unsliced M-step — including a ragged last slice
    and slices past V (V = 100 over 4 shards of 64 rows)."""
    rng = np.random.default_rng(40 + V)
    corpus = random_corpus(rng, 300, V, 1, 40, empty_every=17)
    h1, d1 = _train(ctx, corpus, k, dtype, 6)
    monkeypatch.setenv("STC_VIRTUAL_SHARDS", str(shards))
    h2, d2 = _train(ctx, corpus, k, dtype, 6)
    assert h1.iteration() == h2.iteration() > 0
    np.testing.assert_array_equal(h1.topics(), h2.topics())
    np.testing.assert_array_equal(h1.alpha(), h2.alpha())
    assert h1.bound(d1, gamma_seed=3) == h2.bound(d2, gamma_seed=3)
    np.testing.assert_array_equal(h1.topic_distribution(d1, gamma_seed=3), h2.topic_distribution(d2, gamma_seed=3))


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_prefetched_draws_match_synchronous(ctx, dtype):
    """next() samples draw d+1 during step d and counts it with step d's collective; dropping the
    prefetch before every step (set_corpus) samples each draw synchronously: identical models."""
    rng = np.random.default_rng(44)
    corpus = random_corpus(rng, 500, 2048, 1, 60, empty_every=11)
    h1, _ = _train(ctx, corpus, 8, dtype, 7)
    h2, _ = _train(ctx, corpus, 8, dtype, 7, reset_each=True)
    assert h1.iteration() == h2.iteration() == 7
    np.testing.assert_array_equal(h1.topics(), h2.topics())
    np.testing.assert_array_equal(h1.alpha(), h2.alpha())


def test_empty_draws_advance(ctx):
    """Spark's next() draws a new sample on every call: an empty batch returns without an iteration
    (`if (batch.isEmpty()) return this`), and the following call samples afresh — a 4-doc corpus at
    fraction 0.05 is empty most of the time, yet iterations accrue."""
    rng = np.random.default_rng(45)
    corpus = random_corpus(rng, 4, 256, 5, 20)
    h, _ = _handle(ctx, corpus, 3, "f64", None, mini_batch_fraction=0.05, seed=2)
    h.init_random(1)
    sizes = [h.next()["batch_docs"] for _ in range(200)]
    nonempty = sum(1 for x in sizes if x > 0)
    assert 5 <= nonempty <= 60, nonempty  # Poisson(0.2) over 200 draws: mean ≈ 36
    assert h.iteration() == nonempty


def test_slot_order_longest_first_same_model(ctx, monkeypatch):
    """next() runs a small minibatch's documents longest-first (order_slots: batch / orig / nnz
    permuted together, γ₀ keyed by the member index); the model equals the sampling-order run up
    to sstats' summation order within a term."""
    rng = np.random.default_rng(46)
    corpus = random_corpus(rng, 600, 3000, 1, 120, empty_every=23)
    runs = []
    for sort in ("0", "1"):
        monkeypatch.setenv("STC_SORT_DOCS", sort)
        h, _ = _train(ctx, corpus, 10, "f64", 5)
        runs.append((h.topics(), h.alpha(), h.iteration()))
    (l0, a0, i0), (l1, a1, i1) = runs
    assert i0 == i1 == 5
    np.testing.assert_allclose(l1, l0, rtol=1e-10, atol=0)
    np.testing.assert_allclose(a1, a0, rtol=1e-10, atol=0)


@pytest.mark.parametrize("with_replacement", [False, True])
def test_init_random_and_next_match_oracle(ctx, oracle, with_replacement):
    """A5 + A6 exactly: stc_lda_init_random's λ₀ (oracle.init_lambda), next()'s device-sampled
    membership (oracle.sample_members: Bernoulli / Poisson per doc, the draw counter advancing per
    call) and the counter-RNG γ₀ of each member (oracle.gamma_init keyed by train_doc_key), then three
    next() calls vs three oracle submit_minibatch calls on those members: λ and α to 1e-9 (fp64)."""
    rng = np.random.default_rng(21)
    D, V, k, f, seed = 240, 700, 12, 0.1, 77
    corpus = random_corpus(rng, D, V, 1, 40, empty_every=17)
    h, _ = _handle(ctx, corpus, k, "f64", None, mini_batch_fraction=f, seed=seed,
                   sample_with_replacement=with_replacement, optimize_doc_concentration=True)
    h.init_random(seed)
    lam0 = oracle.init_lambda(seed, V, k)
    np.testing.assert_allclose(h.topics(), lam0, rtol=1e-14)
    assert abs(lam0.mean() - 1.0) < 0.01 and abs(lam0.var() - 0.01) < 0.002  # Gamma(100, 1/100)
    alpha, eta = oracle.resolve_alpha_eta(k)
    state = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=D,
                                  mini_batch_fraction=f, optimize_doc_concentration=True)
    for draw in (1, 2, 3):
        members = oracle.sample_members(seed, draw, 0, D, f, with_replacement)
        assert members, draw
        st = h.next()
        assert st["batch_docs"] == len(members), (draw, st["batch_docs"], len(members))
        it = state.iteration + 1
        g0 = [oracle.gamma_init(seed, oracle.train_doc_key(it, 0, pos), k) for pos in range(len(members))]
        oracle.submit_minibatch(state, [corpus.row(d) for d in members], g0)
    np.testing.assert_allclose(h.topics(), state.lam.T, rtol=1e-9)
    np.testing.assert_allclose(h.alpha(), state.alpha, rtol=1e-9)


@pytest.mark.parametrize("dtype,k", [("f64", 300), ("f32", 1500)])
def test_team_estep_many_documents(ctx, dtype, k, monkeypatch):
    """The team kernel over many documents of uneven length (teams finish documents at different
    times, so the epoch flags and the parity-buffered partials are exercised across hundreds of
    exchanges per team) vs the one-CU many-topic kernel on the same inputs: γ agrees to summation-order
    rounding and the iteration counts match (a doc on the stop rule's boundary may differ by one)."""
    rng = np.random.default_rng(23 + k)
    D, V = 1200, 4096
    corpus = random_corpus(rng, D, V, 100, 500, empty_every=97)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    out = {}
    for P in ("1", "2", "3", "4"):
        monkeypatch.setenv("STC_WIDE_TEAM", P)
        h, _ = _handle(ctx, corpus, k, dtype, lam)
        out[P] = h.estep(np.arange(D), g0, want_stat=True)
    g1, s1, i1 = out["1"]
    for P in ("2", "3", "4"):
        g, st, it = out[P]
        same = it == i1
        if dtype == "f64":
            assert (~same).sum() <= 3, (P, np.flatnonzero(~same))
        else:  # fp32 rounding moves the stop crossing of a few percent of the documents
            assert np.abs(it.astype(int) - i1).max() <= 3 and (~same).mean() < 0.05, (P, np.flatnonzero(~same))
        if dtype == "f64":
            big = g1[same] >= 1.0
            np.testing.assert_allclose(g[same][big], g1[same][big], rtol=1e-9)
        else:  # fp32: the oracle test's per-document bound (summation order moves small topics)
            l1 = np.abs(g[same] - g1[same]).sum(axis=1)
            assert np.all(l1 <= 1e-3 * k + 1e-4 * g1[same].sum(axis=1)), (P, l1.max())
        np.testing.assert_allclose(st.sum(), s1.sum(), rtol=1e-6)


@pytest.mark.parametrize("k", [300, 700])
def test_team_timeout_falls_back_to_the_one_cu_kernel(ctx, k, monkeypatch):
    """A team member that never publishes (debug knob STC_TEAM_FAULT=1, team forced to P = 2; k = 300
    splits rows, k = 700 topics) makes its partner give up.  The SAME call re-runs the slots on the one-CU
    kernel and returns OK: λ, α and γ are bit-identical to a run that used the one-CU kernel from the start
    (STC_WIDE_TEAM=1), for a training step and for topicDistribution."""
    rng = np.random.default_rng(31 + k)
    D, V = 48, 2048
    corpus = random_corpus(rng, D, V, 100, 300)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    ids = np.arange(D)

    def run(team, fault):
        monkeypatch.setenv("STC_WIDE_TEAM", str(team))
        if fault:
            monkeypatch.setenv("STC_TEAM_FAULT", "1")
        else:
            monkeypatch.delenv("STC_TEAM_FAULT", raising=False)
        h, d = _handle(ctx, corpus, k, "f64", lam)
        h.step(ids, g0)
        h.step(ids, g0)
        td = h.topic_distribution(d, gamma0=g0)
        out = (h.topics(), h.alpha(), h.iteration(), td)
        h.close()
        d.free()
        return out

    one = run(1, False)
    fb = run(2, True)
    np.testing.assert_array_equal(fb[0], one[0])
    np.testing.assert_array_equal(fb[1], one[1])
    assert fb[2] == one[2] == 2
    np.testing.assert_array_equal(fb[3], one[3])
    team = run(2, False)  # the healthy team agrees with the one-CU kernel to rounding
    np.testing.assert_allclose(team[0], one[0], rtol=1e-9)


def test_topic_team_lds_layout_follows_the_longest_document(ctx, monkeypatch):
    """k_estep_wide_tc sizes its per-row LDS arrays by the launch's longest document (WideTeam::max_row:
    known for an uploaded CSR, unknown — 512 rows — for a device-built one), so the two layouts keep
    different numbers of block rows in LDS and stream the rest.  The same documents through both give
    bit-identical γ, iteration counts and sufficient statistics (the rows' values and summation order do
    not depend on where a row is kept)."""
    import stc

    rng = np.random.default_rng(2026)
    k, V, D = 1100, 1 << 12, 240
    words = [f"w{i}" for i in range(3000)]
    docs = []
    for _ in range(D):
        pick = rng.choice(len(words), size=int(rng.integers(30, 61)), replace=False)
        docs.append([words[i] for i in pick for _ in range(int(rng.integers(1, 4)))])
    d_dev = stc.HashingTF(numFeatures=V, ctx=ctx).transform_device(docs)  # max_row unknown
    host = d_dev.download()
    assert np.diff(host.indptr).max() > 39  # rows past 24 VGPR + 15 LDS rows: the layouts differ
    d_up = stc.DeviceCsr.upload(ctx, host, stc.STC_F64)  # max_row known
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    monkeypatch.setenv("STC_WIDE_TEAM", "2")
    out = []
    for d in (d_dev, d_up):
        h = stc.LdaHandle(ctx, k, V, dtype="f64")
        h.set_corpus(d, D)
        h.set_topics(lam)
        out.append(h.estep(np.arange(D), g0, want_stat=True))
        assert h.counters()["kernels"]["k_estep_wide_tc"] >= 1
        h.close()
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
    d_dev.free()
    d_up.free()


@pytest.mark.parametrize("k", [20, 100])
def test_presorted_sstats_pairs_bitwise(ctx, monkeypatch, k):
    """fp64 rows path: the (term, slot) pairs built from the batch and radix-sorted beside the E-step
    (STC_PRESORT, the default) give the model of the pairs the E-step writes and sorts after it —
    bit for bit, over sampled next() steps with empty, short and 7–8-row-set documents."""
    rng = np.random.default_rng(47 + k)
    corpus = random_corpus(rng, 400, 4096, 0, 250, empty_every=19)
    runs = []
    for presort in ("0", "1"):
        monkeypatch.setenv("STC_PRESORT", presort)
        h, _ = _train(ctx, corpus, k, "f64", 5)
        runs.append((h.topics(), h.alpha(), h.iteration()))
    (l0, a0, i0), (l1, a1, i1) = runs
    assert i0 == i1 == 5
    np.testing.assert_array_equal(l1, l0)
    np.testing.assert_array_equal(a1, a0)
