"""libstc's own RCCL paths with two ranks (the gloo tests in test_distributed.py only run
the oracle's decomposition).  Two worker processes (tests/comm_worker.py) join one communicator
through stc_comm_init and run stc_lda_next steps, stc_idf_fit and stc_lda_bound; rank 1 holds 4
docs, so its Poisson(0.08) sample is empty in most steps while rank 0's is not — the case where a
per-rank early return used to leave the ranks' collectives unpaired.

Checked: both ranks end with bitwise-identical λ, α and iteration counters, and λ/α equal the
single-process oracle replaying the same device-sampled membership (k_sample's Poisson draw and the
γ₀ keys are restated below) to 1e-9; IDF df/m equal the oracle's over the union of the shards.
"""
import math
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import comm_worker as W  # noqa: E402


def _members(indptr, fraction, seed, iteration, rank, oracle):
    """k_sample (lda.hip): Poisson(f) count per doc from doc_stream(seed ^ 0x5DEECE66D, key)."""
    out = []
    D = indptr.size - 1
    for d in range(D):
        st = oracle.doc_stream(seed ^ 0x5DEECE66D, oracle.train_doc_key(iteration, rank, d))
        u = oracle._uniform(st, 0)
        p = math.exp(-fraction)
        F, c = p, 0
        while u > F and c < 64:
            c += 1
            p *= fraction / c
            F += p
        out += [d] * c
    return out


def test_two_ranks_lda_next_idf_bound(tmp_path, oracle):
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "comm_worker.py"), str(r), "2", str(tmp_path)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("comm workers timed out (unpaired collectives?)")
        logs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    res = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(2)]
    if "comm_error" in res[0] or "comm_error" in res[1]:
        pytest.skip(f"RCCL communicator with two ranks on one device refused: {res[0].get('comm_error')}")
    a, b = res
    # identical replicas
    assert np.array_equal(a["lam"], b["lam"]) and np.array_equal(a["alpha"], b["alpha"])
    assert np.array_equal(a["iters"], b["iters"])
    assert float(a["bound"]) == float(b["bound"]) and float(a["token_count"]) == float(b["token_count"])
    # IDF over the union of the shards
    c0, c1 = W.comm_corpus(0), W.comm_corpus(1)
    ip = np.concatenate([c0.indptr, c1.indptr[1:] + c0.indptr[-1]])
    ix = np.concatenate([c0.indices, c1.indices])
    vv = np.concatenate([c0.values, c1.values])
    idf_o, df_o, m_o = oracle.idf_fit(ip, ix, vv, W.V, 2)
    assert int(a["m"]) == m_o == int(b["m"]) and np.array_equal(a["df"], df_o) and np.array_equal(b["df"], df_o)
    np.testing.assert_allclose(a["idf"], idf_o, rtol=1e-15, atol=0)
    # single-process oracle replay of the sampled membership (global batch = rank 0's then rank 1's)
    total = c0.num_rows + c1.num_rows
    lam0 = np.random.default_rng(9).gamma(100.0, 0.01, size=(W.V, W.K))
    alpha, eta = oracle.resolve_alpha_eta(W.K)
    st = oracle.OnlineLDAState(lam=lam0.T.copy(), alpha=alpha, eta=eta, corpus_size=total,
                               mini_batch_fraction=W.FRACTION, optimize_doc_concentration=True)
    empty_rank1 = 0
    # next_impl (api.hip): the membership is keyed by the DRAW counter, which advances on every call
    # (Spark's generator advances on empty batches too); γ₀ by the iteration the batch would make
    for draw in range(1, W.STEPS + 1):
        it = st.iteration + 1
        docs, g0 = [], []
        for r, c in enumerate((c0, c1)):
            mem = _members(c.indptr, W.FRACTION, W.SEED, draw, r, oracle)
            empty_rank1 += (r == 1 and not mem)
            for pos, d in enumerate(mem):
                docs.append(c.row(d))
                g0.append(oracle.gamma_init(W.SEED, oracle.train_doc_key(it, r, pos), W.K))
        if not docs:  # Spark: the global batch is empty → no iteration
            continue
        oracle.submit_minibatch(st, docs, g0)
    assert empty_rank1 > 0, "the test needs steps where only rank 1's sample is empty"
    assert int(a["iters"][-1]) == st.iteration
    rel = np.max(np.abs(a["lam"] - st.lam.T) / st.lam.T)
    assert rel < 1e-9, rel
    np.testing.assert_allclose(a["alpha"], st.alpha, rtol=1e-9)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_one_rank_communicator_collective_paths(ctx, monkeypatch, dtype):
    """libstc's RCCL calls on a real communicator (one rank: the box has one GPU, and RCCL refuses two
    ranks on one device): with STC_COLLECTIVE_MSTEP=1 every next() runs the multi-GPU M-step — the
    grouped reduce-scatter of stat + all-reduce of logphat/count + the next draw's size, the sliced λ
    update, the colsum-partial all-gather, the expElogβ'/logscale all-gathers — then get_topics
    gathers the sharded λ and the bound all-reduces its corpus and topics parts; IDF fit reduces
    df/m.  Everything must be bit-identical to the same run without a communicator."""
    import stc
    from helpers import random_corpus

    rng = np.random.default_rng(51)
    corpus = random_corpus(rng, 400, 3000, 1, 50, empty_every=9)
    c1 = stc.Context(0)
    c1.comm_init(stc.Context.unique_id(), 1, 0)
    dt = stc.STC_F32 if dtype == "f32" else stc.STC_F64
    runs = []
    for c, coll in ((ctx, "0"), (c1, "1")):
        monkeypatch.setenv("STC_COLLECTIVE_MSTEP", coll)
        h = stc.LdaHandle(c, 9, corpus.num_cols, mini_batch_fraction=0.2, seed=4, dtype=dtype,
                          optimize_doc_concentration=True)
        d = stc.DeviceCsr.upload(c, corpus, dt)
        h.set_corpus(d, corpus.num_rows)
        h.init_random(6)
        for _ in range(6):
            h.next(stats=False)
        bound = h.bound(d, gamma_seed=2)  # before get_topics: λ still sharded, topics part all-reduced
        idf = stc.IDF(minDocFreq=2, ctx=c).fit(corpus)
        runs.append(dict(lam=h.topics(), alpha=h.alpha(), it=h.iteration(), bound=bound, idf=idf.idf,
                         df=idf.docFreq))
    a, b = runs
    assert a["it"] == b["it"] == 6
    np.testing.assert_array_equal(a["lam"], b["lam"])
    np.testing.assert_array_equal(a["alpha"], b["alpha"])
    assert a["bound"] == b["bound"]
    np.testing.assert_array_equal(a["idf"], b["idf"])
    np.testing.assert_array_equal(a["df"], b["df"])
