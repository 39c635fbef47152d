"""GPU: the single-process multi-device handle (stc_group — SURVEY.md §8(b); the JVM drop-in's multi-GPU
form) against a single handle on the same inputs.

The box has one GPU, so the groups here repeat device 0: the members run the multi-GPU decomposition
(document shards, the stat reduce-scatter, the vocabulary-sliced λ update, the colsum / expElogβ' /
logscale all-gathers, the sharded bound) on one device through the in-process transport — the same call
sequence RCCL carries between distinct devices.  A one-member group is the plain single-GPU path.
Tolerances: fp64, only the summation order of sstats across shards differs (1e-12 relative on λ)."""
import numpy as np
import pytest

from helpers import long_run_corpus, random_corpus

pytestmark = pytest.mark.gpu


def _single(ctx, corpus, k, lam, **kw):
    import stc

    h = stc.LdaHandle(ctx, k, corpus.num_cols, dtype="f64", **kw)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h.set_corpus(d, corpus.num_rows)
    h.set_topics(lam)
    return h, d


@pytest.mark.parametrize("members", [1, 2, 3, 4])
def test_group_steps_match_a_single_handle(ctx, members):
    """Injected membership (global ids, duplicates included) and γ₀: λ, α and the iteration count after
    three steps; then describeTopics, the bound and topicDistribution over held-out rows."""
    import stc

    rng = np.random.default_rng(100 + members)
    D, V, k = 240, 3000, 40
    corpus = random_corpus(rng, D, V, 1, 160, empty_every=17)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    kw = dict(mini_batch_fraction=0.3, optimize_doc_concentration=True)
    h, d = _single(ctx, corpus, k, lam, **kw)
    with stc.LdaGroup([0] * members, k, V, dtype="f64", **kw) as g:
        g.set_corpus(corpus)
        g.set_topics(lam)
        for it in range(3):
            ids = rng.integers(0, D, size=90)
            g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
            sh = h.step(ids, g0)
            sg = g.step(ids, g0)
            assert sg["batch_docs"] == sh["batch_docs"] and sg["nonempty_docs"] == sh["nonempty_docs"]
            # step 1 starts from the same λ (identical per-document E-steps); later steps from λ that
            # differs in the last bits (stat summed in shard order), where a document on the stop rule's
            # boundary may take one more or one fewer iteration
            assert abs(sg["inner_iters"] - sh["inner_iters"]) <= (0 if it == 0 else 2)
        np.testing.assert_allclose(g.topics(), h.topics(), rtol=1e-12)
        np.testing.assert_allclose(g.alpha(), h.alpha(), rtol=1e-12)
        assert g.iteration() == h.iteration() == 3
        ig, wg = g.describe(10)
        ih, wh = h.describe(10)
        assert np.array_equal(ig, ih)
        np.testing.assert_allclose(wg, wh, rtol=1e-12)
        held = random_corpus(rng, 70, V, 0, 120, empty_every=11)
        dh = stc.DeviceCsr.upload(ctx, held, stc.STC_F64)
        bh = h.bound(dh, gamma_seed=7, doc_id_base=1000)
        bg = g.bound(held, gamma_seed=7, doc_id_base=1000)
        np.testing.assert_allclose(bg["bound"], bh["bound"], rtol=1e-11)
        assert bg["token_count"] == bh["token_count"]
        np.testing.assert_allclose(g.topic_distribution(held, gamma_seed=7, doc_id_base=1000),
                                   h.topic_distribution(dh, gamma_seed=7, doc_id_base=1000), rtol=1e-10, atol=1e-14)
        dh.free()


def test_group_next_trains_every_member(ctx):
    """next(): each member samples its own shard; the global batch, the shared λ and α move together."""
    import stc

    rng = np.random.default_rng(3)
    D, V, k = 400, 2048, 24
    corpus = random_corpus(rng, D, V, 1, 100)
    with stc.LdaGroup([0, 0, 0], k, V, dtype="f64", mini_batch_fraction=0.2, seed=11) as g:
        g.set_corpus(corpus)
        g.init_random(11)
        lam0 = g.topics()
        total = 0
        for _ in range(4):
            st = g.next()
            total += st["batch_docs"]
        assert g.iteration() == 4 and total > 0.1 * 4 * D
        assert not np.array_equal(g.topics(), lam0)
        assert np.all(np.isfinite(g.topics())) and np.all(g.alpha() > 0)


def _shard_rows(indptr, n):
    """stc_group's document split (api.hip shard_rows): contiguous rows, nnz-balanced."""
    rows, nnz = indptr.size - 1, int(indptr[-1])
    r0, r = [0], 0
    for q in range(1, n):
        target = (nnz * q + n - 1) // n
        while r < rows and indptr[r] < target:
            r += 1
        r0.append(max(r, r0[-1]))
    return r0 + [rows]


@pytest.mark.parametrize("members", [2, 3])
def test_group_next_matches_the_oracle_replay(ctx, oracle, members):
    """The multi-rank sharded path end to end (per-member Poisson draws keyed by (draw, rank, local row),
    the global-empty rule, the sliced λ update and its all-gathers) against the single-process oracle
    replaying the same membership (test_gpu_comm._members restates k_sample).  fp64, 1e-9 on λ and α."""
    import stc
    from test_gpu_comm import _members

    rng = np.random.default_rng(70 + members)
    D, V, k, seed, frac, steps = 90, 700, 6, 77, 0.05, 8
    corpus = random_corpus(rng, D, V, 1, 30, empty_every=11)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    r0 = _shard_rows(corpus.indptr, members)
    with stc.LdaGroup([0] * members, k, V, dtype="f64", mini_batch_fraction=frac, seed=seed,
                      optimize_doc_concentration=True) as g:
        g.set_corpus(corpus)
        g.set_topics(lam0)
        for _ in range(steps):
            g.next()
        lam, alpha, iters = g.topics(), g.alpha(), g.iteration()
    alpha0, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha0, eta=eta, corpus_size=D, mini_batch_fraction=frac,
                               optimize_doc_concentration=True)
    empty = 0
    for draw in range(1, steps + 1):
        it = st.iteration + 1
        docs, g0 = [], []
        for r in range(members):
            lo, hi = r0[r], r0[r + 1]
            ip = corpus.indptr[lo:hi + 1] - corpus.indptr[lo]
            for pos, dl in enumerate(_members(ip, frac, seed, draw, r, oracle)):
                docs.append(corpus.row(lo + dl))
                g0.append(oracle.gamma_init(seed, oracle.train_doc_key(it, r, pos), k))
        if not docs:
            empty += 1
            continue
        oracle.submit_minibatch(st, docs, g0)
    assert iters == st.iteration and st.iteration > 0
    rel = np.max(np.abs(lam - st.lam.T) / st.lam.T)
    assert rel < 1e-9, rel
    np.testing.assert_allclose(alpha, st.alpha, rtol=1e-9)


def test_group_argument_errors(ctx):
    import stc

    with pytest.raises(stc.StcIllegalArgument):
        stc.LdaGroup([0, 99], 8, 100)
    with pytest.raises(stc.StcIllegalArgument):
        stc.LdaGroup([], 8, 100)


def test_failed_set_corpus_leaves_every_member_on_its_shard(ctx, monkeypatch):
    """member 1's upload of a new corpus fails (debug knob STC_GROUP_UPLOAD_FAULT=1).  The
    call raises, no member was switched to the new shards (freed again), and training continues on the
    previous corpus exactly as a group that never saw the failed call; also timing / counters per member."""
    import stc

    rng = np.random.default_rng(77)
    D, V, k = 200, 2500, 24
    corpus = random_corpus(rng, D, V, 1, 140)
    other = random_corpus(rng, 150, V, 1, 90)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    ids = [rng.integers(0, D, size=60) for _ in range(2)]
    g0 = [rng.gamma(100.0, 0.01, size=(60, k)) for _ in range(2)]

    def run(fail):
        with stc.LdaGroup([0, 0], k, V, dtype="f64") as g:
            g.set_corpus(corpus)
            g.set_topics(lam)
            g.step(ids[0], g0[0])
            if fail:
                monkeypatch.setenv("STC_GROUP_UPLOAD_FAULT", "1")
                with pytest.raises(stc.StcError, match="injected shard upload failure"):
                    g.set_corpus(other)
                monkeypatch.delenv("STC_GROUP_UPLOAD_FAULT")
            g.enable_timing(True)
            g.step(ids[1], g0[1])
            g.next(stats=False)
            g.synchronize()
            cs = g.counters()
            assert len(cs) == 2 and sum(c["docs"] for c in cs) > 0
            assert all(p["estep"] >= 0.0 for p in g.phase_times())
            t, a = g.topics(), g.alpha()
            # the model handed to inference drops its corpus shards: describe still works, training does not
            g.release_corpus()
            idx, _ = g.describe(5)
            assert idx.shape == (k, 5)
            with pytest.raises(stc.StcError, match="corpus"):
                g.next(stats=False)
            return t, a

    t0, a0 = run(False)
    t1, a1 = run(True)
    np.testing.assert_array_equal(t1, t0)
    np.testing.assert_array_equal(a1, a0)


# ---- the group's RCCL path (ncclCommInitAll + one host thread per member) on a one-GPU box.
# STC_GROUP_RCCL=1: a group of distinct devices — here the one device — builds a real communicator with
# ncclCommInitAll, runs the sliced (multi-rank) M-step's reduce-scatter / all-reduce / all-gathers over it
# and drives its member from a spawned host thread, exactly as configs[2]'s one-JVM, N-GPU drop-in does.

def test_rccl_group_matches_a_single_handle(ctx, monkeypatch):
    """Injected membership and γ₀ through a one-member RCCL group: λ, α, iteration count, describeTopics,
    the bound and topicDistribution bit-identical to a plain single handle (a one-rank reduce-scatter /
    all-gather is a copy and the slice is the whole vocabulary)."""
    import stc

    monkeypatch.setenv("STC_GROUP_RCCL", "1")
    rng = np.random.default_rng(211)
    D, V, k = 240, 3000, 40
    corpus = random_corpus(rng, D, V, 1, 160, empty_every=17)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    kw = dict(mini_batch_fraction=0.3, optimize_doc_concentration=True)
    h, d = _single(ctx, corpus, k, lam, **kw)
    with stc.LdaGroup([0], k, V, dtype="f64", **kw) as g:
        assert g.transport() == "rccl"
        g.set_corpus(corpus)
        g.set_topics(lam)
        for _ in range(3):
            ids = rng.integers(0, D, size=90)
            g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
            sh, sg = h.step(ids, g0), g.step(ids, g0)
            assert sg["inner_iters"] == sh["inner_iters"] and sg["nonempty_docs"] == sh["nonempty_docs"]
        np.testing.assert_array_equal(g.topics(), h.topics())
        np.testing.assert_array_equal(g.alpha(), h.alpha())
        assert g.iteration() == h.iteration() == 3
        ig, wg = g.describe(10)
        ih, wh = h.describe(10)
        assert np.array_equal(ig, ih) and np.array_equal(wg, wh)
        held = random_corpus(rng, 70, V, 0, 120, empty_every=11)
        dh = stc.DeviceCsr.upload(ctx, held, stc.STC_F64)
        assert g.bound(held, gamma_seed=7, doc_id_base=1000)["bound"] == h.bound(dh, gamma_seed=7, doc_id_base=1000)["bound"]
        np.testing.assert_array_equal(g.topic_distribution(held, gamma_seed=7, doc_id_base=1000),
                                      h.topic_distribution(dh, gamma_seed=7, doc_id_base=1000))
        dh.free()
        # device-sampled next() through the same communicator, then the sharded λ gathered back
        g.next()
        g.next(stats=False)
        g.synchronize()
        assert g.iteration() == 5 and np.all(np.isfinite(g.topics()))


def test_rccl_group_next_matches_the_oracle_replay(ctx, oracle, monkeypatch, dtype="f64"):
    """The device-sampled next() path over the real communicator against the single-process oracle replaying
    the same membership (as test_group_next_matches_the_oracle_replay for the in-process transport)."""
    import stc
    from test_gpu_comm import _members

    monkeypatch.setenv("STC_GROUP_RCCL", "1")
    rng = np.random.default_rng(170)
    D, V, k, seed, frac, steps = 90, 700, 6, 77, 0.05, 8
    corpus = random_corpus(rng, D, V, 1, 30, empty_every=11)
    lam0 = rng.gamma(100.0, 0.01, size=(V, k))
    with stc.LdaGroup([0], k, V, dtype=dtype, mini_batch_fraction=frac, seed=seed,
                      optimize_doc_concentration=True) as g:
        assert g.transport() == "rccl"
        g.set_corpus(corpus)
        g.set_topics(lam0)
        for _ in range(steps):
            g.next()
        lam, alpha, iters = g.topics(), g.alpha(), g.iteration()
    alpha0, eta = oracle.resolve_alpha_eta(k)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha0, eta=eta, corpus_size=D, mini_batch_fraction=frac,
                               optimize_doc_concentration=True)
    for draw in range(1, steps + 1):
        it = st.iteration + 1
        mem = _members(corpus.indptr, frac, seed, draw, 0, oracle)
        if not mem:
            continue
        oracle.submit_minibatch(st, [corpus.row(dd) for dd in mem],
                                [oracle.gamma_init(seed, oracle.train_doc_key(it, 0, pos), k) for pos in range(len(mem))])
    assert iters == st.iteration and st.iteration > 0
    rel = np.max(np.abs(lam - st.lam.T) / st.lam.T)
    assert rel < 1e-9, rel
    np.testing.assert_allclose(alpha, st.alpha, rtol=1e-9)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_rccl_group_next_bitwise_equals_the_plain_group(ctx, monkeypatch, dtype):
    """next() steps through the one-member RCCL group (sliced M-step, collectives, member thread) are
    bit-identical to the same steps through a plain one-member group, in both dtypes."""
    import stc

    rng = np.random.default_rng(5)
    D, V, k = 400, 3000, 9
    corpus = random_corpus(rng, D, V, 1, 50, empty_every=9)
    runs = []
    for knob in ("0", "1"):
        monkeypatch.setenv("STC_GROUP_RCCL", knob)
        with stc.LdaGroup([0], k, V, dtype=dtype, mini_batch_fraction=0.2, seed=4,
                          optimize_doc_concentration=True) as g:
            assert g.transport() == ("rccl" if knob == "1" else "none")
            g.set_corpus(corpus)
            g.init_random(6)
            for _ in range(6):
                g.next(stats=False)
            runs.append((g.topics(), g.alpha(), g.iteration()))
    (t0, a0, i0), (t1, a1, i1) = runs
    assert i0 == i1 == 6
    np.testing.assert_array_equal(t1, t0)
    np.testing.assert_array_equal(a1, a0)


def test_group_transport_kinds(ctx, monkeypatch):
    import stc

    monkeypatch.delenv("STC_GROUP_RCCL", raising=False)
    with stc.LdaGroup([0], 8, 100) as g:
        assert g.transport() == "none"
    with stc.LdaGroup([0, 0], 8, 100) as g:
        assert g.transport() == "in-process"


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_chunked_reduce_scatter_is_bitwise_the_single_one(ctx, monkeypatch, dtype):
    """The sharded step with the stat reduce-scatter split into vocabulary sub-chunks (api.hip
    train_tail_split: one sstats launch per sub-chunk, each sub-chunk's reduce-scatter on the collective
    stream under the next sstats launch, the M-step of sub-chunk j under the reduce-scatter of j+1)
    against STC_RS_CHUNKS=1 (one reduce-scatter after the whole stat): λ, α, expElogβ'-dependent
    topicDistribution and the step statistics bit-identical over sampled steps (next(): the draw-count
    all-reduce rides on sub-chunk 0) and injected ones.  V = 5000 over 3 members: 27 blocks of 64 rows
    per slice, cut 7+7+7+6 (STC_RS_CHUNKS=4) and 6+6+6+6+3 (=5)."""
    import stc

    rng = np.random.default_rng(31)
    D, V, k = 400, 5000, 24
    corpus = random_corpus(rng, D, V, 1, 120, empty_every=13)
    ids = rng.integers(0, D, size=150)
    g0 = rng.gamma(100.0, 0.01, size=(ids.size, k))
    out = {}
    for chunks in ("1", "4", "5"):
        monkeypatch.setenv("STC_RS_CHUNKS", chunks)
        with stc.LdaGroup([0, 0, 0], k, V, dtype=dtype, mini_batch_fraction=0.25, seed=8,
                          optimize_doc_concentration=True) as g:
            g.set_corpus(corpus)
            g.init_random(3)
            stats = [g.next() for _ in range(3)]
            stats.append(g.step(ids, g0))
            td = g.topic_distribution(corpus)
            out[chunks] = (g.topics(), g.alpha(), td, stats)
    ref = out["1"]
    for chunks in ("4", "5"):
        got = out[chunks]
        for a, b in zip(got[:3], ref[:3]):
            np.testing.assert_array_equal(a, b)
        assert got[3] == ref[3]


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_chunked_reduce_scatter_long_runs(ctx, monkeypatch, dtype):
    """The sub-chunk sstats launches (StatMap) where frequent terms' runs span full 32-chunk tiles in
    every member (lda.hip k_fixup_tiles: a sub-chunk launch sums only its own terms' tiles): an injected
    step of 60000 documents over 3 members, hot terms in slices 0, 1 and 2 and in several sub-chunks,
    STC_RS_CHUNKS=4 bit-identical to the single reduce-scatter."""
    import stc

    rng = np.random.default_rng(32)
    D, V, k = 60000, 5000, 24
    corpus = long_run_corpus(rng, D, V, [0, 1, 1500, 3100, 4900, 4999])
    ids = np.arange(D)
    g0 = rng.gamma(100.0, 0.01, size=(D, k))
    out = {}
    for chunks in ("1", "4"):
        monkeypatch.setenv("STC_RS_CHUNKS", chunks)
        with stc.LdaGroup([0, 0, 0], k, V, dtype=dtype, seed=8, optimize_doc_concentration=True) as g:
            g.set_corpus(corpus)
            g.init_random(3)
            st = g.step(ids, g0)
            out[chunks] = (g.topics(), g.alpha(), st)
    for a, b in zip(out["4"][:2], out["1"][:2]):
        np.testing.assert_array_equal(a, b)
    assert out["4"][2] == out["1"][2]


# ---- the RCCL group is fail-safe before the first multi-GPU run.  A member that throws
# mid-step leaves its peers' collectives without a partner; the group must abort every communicator
# (ncclCommAbort), report the failure, refuse later calls and still be destroyable, and a stuck wait must
# end at a deadline (STC_COLL_TIMEOUT_MS) instead of hanging the process.

def _destroy_rc(g):
    rc = g.lib.stc_group_destroy(g.handle)
    g.handle = None
    return rc


def test_rccl_group_member_failure_aborts_and_a_new_group_trains_bitwise(ctx, monkeypatch):
    """STC_GROUP_STEP_FAULT=0:3 — the member thread throws on its third step, after E-step + sstats and
    before the reduce-scatter: that call returns the error, the communicator is aborted, every later call
    is STC_ERR_STATE, stc_group_destroy returns 0; then a fresh RCCL group trains bit-identically to a
    plain group (as test_rccl_group_next_bitwise_equals_the_plain_group)."""
    import time

    import stc

    rng = np.random.default_rng(5)
    D, V, k = 400, 3000, 9
    corpus = random_corpus(rng, D, V, 1, 50, empty_every=9)
    monkeypatch.setenv("STC_GROUP_RCCL", "1")
    monkeypatch.setenv("STC_GROUP_STEP_FAULT", "0:3")
    g = stc.LdaGroup([0], k, V, dtype="f64", mini_batch_fraction=0.2, seed=4, optimize_doc_concentration=True)
    assert g.transport() == "rccl"
    g.set_corpus(corpus)
    g.init_random(6)
    g.next()
    g.next(stats=False)
    with pytest.raises(stc.StcError) as e:
        g.next()
    assert e.value.code == stc.STC_ERR_STATE and "STC_GROUP_STEP_FAULT" in str(e.value)
    for call in (g.next, g.topics, g.alpha, g.synchronize):
        with pytest.raises(stc.StcError) as e:
            call()
        assert e.value.code == stc.STC_ERR_STATE and "aborted" in str(e.value)
    assert g.transport() == "rccl"  # (introspection still answers)
    t0 = time.perf_counter()
    assert _destroy_rc(g) == 0
    assert time.perf_counter() - t0 < 30
    monkeypatch.delenv("STC_GROUP_STEP_FAULT")
    runs = []
    for knob in ("0", "1"):
        monkeypatch.setenv("STC_GROUP_RCCL", knob)
        with stc.LdaGroup([0], k, V, dtype="f64", mini_batch_fraction=0.2, seed=4,
                          optimize_doc_concentration=True) as g2:
            g2.set_corpus(corpus)
            g2.init_random(6)
            for _ in range(6):
                g2.next(stats=False)
            runs.append((g2.topics(), g2.alpha(), g2.iteration()))
    (t0_, a0, i0), (t1, a1, i1) = runs
    assert i0 == i1 == 6
    np.testing.assert_array_equal(t1, t0_)
    np.testing.assert_array_equal(a1, a0)


def test_rccl_group_wait_deadline_aborts(ctx, monkeypatch):
    """STC_COLL_TIMEOUT_MS=1: a step whose device work outlasts the deadline ends as STC_ERR_RCCL (the wait
    behind the collectives gave up and aborted the communicator) instead of blocking; the group is then
    refused and destroyable."""
    import stc

    rng = np.random.default_rng(6)
    D, V, k = 20000, 4096, 40
    corpus = random_corpus(rng, D, V, 60, 200)
    monkeypatch.setenv("STC_GROUP_RCCL", "1")
    monkeypatch.setenv("STC_COLL_TIMEOUT_MS", "1")
    g = stc.LdaGroup([0], k, V, dtype="f64", mini_batch_fraction=1.0, seed=4)
    g.set_corpus(corpus)
    g.init_random(6)
    with pytest.raises(stc.StcError) as e:
        for _ in range(3):
            g.next()
    assert e.value.code == stc.STC_ERR_RCCL and "STC_COLL_TIMEOUT_MS" in str(e.value)
    with pytest.raises(stc.StcError) as e:
        g.next()
    assert e.value.code == stc.STC_ERR_STATE
    assert _destroy_rc(g) == 0


def test_rank_communicator_wait_deadline_aborts(monkeypatch):
    """The torchrun "ranks" form (one context per process, stc_comm_init): the same deadline on its waits —
    a step that outlasts STC_COLL_TIMEOUT_MS raises STC_ERR_RCCL, the communicator is aborted, a later step
    is STC_ERR_STATE, and the handle and context still free."""
    import stc

    rng = np.random.default_rng(7)
    D, V, k = 20000, 4096, 40
    corpus = random_corpus(rng, D, V, 60, 200)
    monkeypatch.setenv("STC_COLL_TIMEOUT_MS", "1")
    monkeypatch.setenv("STC_COLLECTIVE_MSTEP", "1")
    c1 = stc.Context(0)
    c1.comm_init(stc.Context.unique_id(), 1, 0)
    h = stc.LdaHandle(c1, k, V, mini_batch_fraction=1.0, seed=4, dtype="f64")
    d = stc.DeviceCsr.upload(c1, corpus, stc.STC_F64)
    h.set_corpus(d, D)
    h.init_random(6)
    with pytest.raises(stc.StcError) as e:
        for _ in range(3):
            h.next()
    assert e.value.code == stc.STC_ERR_RCCL
    with pytest.raises(stc.StcError) as e:
        h.next()
    assert e.value.code == stc.STC_ERR_STATE
    h.close()
    d.free()
    c1.close()
