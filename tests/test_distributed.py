"""World-size-2 (gloo, CPU) tests of the sharded decomposition the library runs over RCCL.

The product shards a minibatch by document.  Each rank:
* runs the E-step on its members;
* accumulates its partial `stat` (V×k), logphat and non-empty count;
* joins a reduce-scatter of `stat` over vocabulary slices of Vs rows (Vs a multiple of the 64-row
  λ-update block) grouped with the all-reduce of logphat / count (api.hip train_tail);
* updates λ on its slice, all-gathers the per-block colsum partials (reduced in block order, so every
  rank holds the same colsum), computes its slice of expElogβ and all-gathers it for the next E-step;
* gathers λ only when a reader asks (gather_lambda); the bound sums each slice's topics part.

IDF reduces df and m the same way (stc_idf_fit), and the bound reduces its corpus part.  These
tests run exactly that decomposition with the oracle's per-document primitives on two gloo ranks.
They check that it reproduces the single-process [U] submitMiniBatch / IDF.fit / logLikelihood,
so the N > 1 data flow is correct by construction before the driver runs it on 8 GPUs.
"""
import math
import os
import socket
import tempfile

import numpy as np
import pytest

from helpers import random_corpus


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem():
    rng = np.random.default_rng(7)
    D, V, k = 48, 96, 5
    corpus = random_corpus(rng, D, V, 0, 30)  # includes empty docs
    lam = rng.gamma(100.0, 0.01, size=(k, V))
    alpha = np.full(k, 1.0 / k)
    batch = np.sort(rng.choice(D, size=30, replace=False))
    g0 = rng.gamma(100.0, 0.01, size=(batch.size, k))
    return corpus, lam, alpha, batch, g0


def _partial_stats(O, lam, alpha, docs, gamma0s):
    """The per-rank half of submitMiniBatch (what estep_and_stats computes on one GPU)."""
    k, V = lam.shape
    eeb = np.exp(O.dirichlet_expectation(lam)).T
    stat = np.zeros((k, V))
    logphat = np.zeros(k)
    n = 0
    for (ids, cts), g0 in zip(docs, gamma0s):
        if len(ids) == 0 or not np.any(np.asarray(cts) != 0):
            continue
        n += 1
        gamma, sstats, _ = O.variational_topic_inference(ids, cts, eeb, alpha, g0)
        np.add.at(stat.T, np.asarray(ids), sstats.T)
        logphat += O.dirichlet_expectation(gamma)
    return stat, logphat, n, eeb


def _worker(rank, world, port, out_dir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from oracle import oracle as O

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    corpus, lam, alpha, batch, g0 = _problem()
    k, V = lam.shape

    # --- one minibatch, members split by contiguous ranges (the library's doc sharding)
    mine = np.array_split(np.arange(batch.size), world)[rank]
    docs = [corpus.row(int(batch[i])) for i in mine]
    stat, logphat, n, eeb = _partial_stats(O, lam, alpha, docs, g0[mine])
    small = torch.from_numpy(np.concatenate([logphat, [float(n)]]))
    # vocabulary slices: Vs = ⌈⌈V/N⌉/64⌉·64 rows per rank, stat padded with zero rows to N·Vs
    RB = 64
    Vs = -(-(-(-V // world)) // RB) * RB
    v0, vn = rank * Vs, max(0, min(V - rank * Vs, Vs))
    st = torch.zeros((world * Vs, k), dtype=torch.float64)
    st[:V] = torch.from_numpy(stat.T)
    mine_st = torch.zeros((Vs, k), dtype=torch.float64)
    dist.reduce_scatter_tensor(mine_st, st)   # ≙ ncclReduceScatter(stat)
    dist.all_reduce(small)                    # ≙ ncclAllReduce(small)  (same group on the GPU)
    logphat_g, n_g = small.numpy()[:k], int(small.numpy()[k])
    # the slice's λ update (the oracle's updateLambda on the slice's columns)
    state = O.OnlineLDAState(lam=lam[:, v0:v0 + vn].copy(), alpha=alpha.copy(), eta=1.0 / k,
                             corpus_size=corpus.num_rows, mini_batch_fraction=batch.size / corpus.num_rows,
                             optimize_doc_concentration=True)
    state.iteration += 1
    O.update_lambda(state, mine_st.numpy()[:vn].T * eeb.T[:, v0:v0 + vn],
                    int(math.ceil(state.mini_batch_fraction * state.corpus_size)))
    O.update_alpha(state, logphat_g / n_g, n_g)
    # colsum: per-64-row-block partials all-gathered, reduced in block order (identical on all ranks)
    lam_slice = np.zeros((k, Vs))
    lam_slice[:, :vn] = state.lam
    part = torch.from_numpy(np.ascontiguousarray(lam_slice.reshape(k, Vs // RB, RB).sum(axis=2).T))
    parts = torch.zeros((world * (Vs // RB), k), dtype=torch.float64)
    dist.all_gather_into_tensor(parts, part)
    colsum = np.zeros(k)
    for b in range(parts.shape[0]):
        colsum += parts[b].numpy()
    # the slice's expElogβ = exp(ψ(λ) − ψ(colsum)), all-gathered (≙ ncclAllGather of Bp)
    eeb_slice = np.zeros((Vs, k))
    eeb_slice[:vn] = np.exp(O.digamma(state.lam) - O.digamma(colsum)[:, None]).T
    eeb_all = torch.zeros((world * Vs, k), dtype=torch.float64)
    dist.all_gather_into_tensor(eeb_all, torch.from_numpy(eeb_slice))
    # a reader's λ (gather_lambda)
    lam_all = torch.zeros((world * Vs, k), dtype=torch.float64)
    dist.all_gather_into_tensor(lam_all, torch.from_numpy(np.ascontiguousarray(lam_slice.T)))
    state.lam = lam_all.numpy()[:V].T.copy()

    # --- IDF: df and m reduced over the ranks (stc_idf_fit with a communicator)
    rows = np.array_split(np.arange(corpus.num_rows), world)[rank]
    lo, hi = corpus.indptr[rows[0]], corpus.indptr[rows[-1] + 1]
    ind, val = corpus.indices[lo:hi], corpus.values[lo:hi]
    df = torch.from_numpy(np.bincount(ind[val > 0], minlength=V).astype(np.int64))
    m = torch.tensor([rows.size], dtype=torch.int64)
    dist.all_reduce(df)
    dist.all_reduce(m)
    mdf = 2
    idf = np.where(df.numpy() >= mdf, np.log((int(m) + 1.0) / (df.numpy() + 1.0)), 0.0)

    # --- bound: corpus part over the rank's documents; topics part: the element sum over the rank's
    # vocabulary slice (λ sharded), both all-reduced, plus the per-topic normaliser once (api.hip
    # topics_part / stc_lda_bound)
    bdocs = [corpus.row(int(r)) for r in rows]
    bg0 = np.stack([O.gamma_init(11, int(r), k) for r in rows])
    _, part, _ = O.log_likelihood_bound(bdocs, bg0, lam.T, alpha, 1.0 / k)
    eta = 1.0 / k
    elog_beta = O.dirichlet_expectation(lam)[:, v0:v0 + vn]   # k × slice, ψ(colsum) of the whole λ
    ls = lam[:, v0:v0 + vn]
    elem = np.sum((eta - ls) * elog_beta) + np.sum(O.gammaln(ls) - O.gammaln(eta))
    cp = torch.tensor([part, elem], dtype=torch.float64)
    dist.all_reduce(cp)
    topics_only = float(cp[1]) + np.sum(O.gammaln(eta * V) - O.gammaln(lam.sum(axis=1)))

    # --- RNG independence of the ranks' γ₀ streams (train_doc_key carries the rank)
    key0 = O.gamma_init(5, O.train_doc_key(3, rank, 0), k)

    # --- the bench's control plane: rank 0's RCCL unique id reaches every rank unchanged
    uid = [bytes(np.random.default_rng(99).integers(0, 256, 128, dtype=np.uint8)) if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)

    np.savez(os.path.join(out_dir, f"r{rank}.npz"), lam=state.lam, alpha=state.alpha, idf=idf,
             eeb=eeb_all.numpy()[:V], colsum=colsum,
             bound=float(cp[0]) + topics_only, key0=key0, uid=np.frombuffer(uid[0], np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_rank_results():
    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        yield [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(2)]


def test_sharded_minibatch_matches_single_process(two_rank_results, oracle):
    O = oracle
    corpus, lam, alpha, batch, g0 = _problem()
    k = lam.shape[0]
    ref = O.OnlineLDAState(lam=lam.copy(), alpha=alpha.copy(), eta=1.0 / k, corpus_size=corpus.num_rows,
                           mini_batch_fraction=batch.size / corpus.num_rows, optimize_doc_concentration=True)
    O.submit_minibatch(ref, [corpus.row(int(b)) for b in batch], g0)
    r0, r1 = two_rank_results
    # λ and α replicated bit-for-bit on both ranks (same reduced inputs, same M-step)
    assert np.array_equal(r0["lam"], r1["lam"]) and np.array_equal(r0["alpha"], r1["alpha"])
    # and equal to the unsharded step up to the reduction's summation order
    np.testing.assert_allclose(r0["lam"], ref.lam, rtol=1e-12, atol=0)
    np.testing.assert_allclose(r0["alpha"], ref.alpha, rtol=1e-12, atol=0)
    # the sharded colsum / expElogβ the next E-step reads: identical on both ranks, and the model's
    assert np.array_equal(r0["colsum"], r1["colsum"]) and np.array_equal(r0["eeb"], r1["eeb"])
    np.testing.assert_allclose(r0["colsum"], ref.lam.sum(axis=1), rtol=1e-13)
    np.testing.assert_allclose(r0["eeb"], np.exp(O.dirichlet_expectation(ref.lam)).T, rtol=1e-12)


def test_sharded_idf_is_bit_exact(two_rank_results, oracle):
    corpus = _problem()[0]
    idf, _, _ = oracle.idf_fit(corpus.indptr, corpus.indices, corpus.values, 96, min_doc_freq=2)
    for r in two_rank_results:
        assert np.array_equal(r["idf"], idf)  # integer df/m reduction ⇒ identical doubles


def test_sharded_bound_matches(two_rank_results, oracle):
    O = oracle
    corpus, lam, alpha, _, _ = _problem()
    k = lam.shape[0]
    docs = [corpus.row(i) for i in range(corpus.num_rows)]
    g0 = np.stack([O.gamma_init(11, i, k) for i in range(corpus.num_rows)])
    ref = O.log_likelihood_bound(docs, g0, lam.T, alpha, 1.0 / k)[0]
    for r in two_rank_results:
        assert abs(float(r["bound"]) - ref) <= 1e-12 * abs(ref)


def test_rank_streams_and_control_plane(two_rank_results):
    r0, r1 = two_rank_results
    assert not np.array_equal(r0["key0"], r1["key0"])  # per-rank γ₀ streams differ
    assert np.array_equal(r0["uid"], r1["uid"])        # uid broadcast intact
