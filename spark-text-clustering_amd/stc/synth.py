"""Seeded synthetic Zipfian corpora of the BASELINE.json shapes.

* ``zipf``     — every token's frequency rank r ~ Zipf(s) over V, term id = π(r) for a seeded
                 permutation π (hot terms scattered over the id space, as hashing does).
* ``zipf-lda`` — the same marginal shape drawn through an LDA generative model: k topics, each a
                 Zipf(s) over its own permutation; θ_d ~ Dir(α0); z ~ θ_d; w = π_z(r).  This gives
                 the topical structure an LDA fit converges on (warm E-step state).
Counts are multiplicities; rows are sorted unique ids (Spark SparseVector semantics).
"""
from __future__ import annotations

import numpy as np

from .core import CsrMatrix


def _zipf_cdf(V, s):
    w = 1.0 / np.power(np.arange(1, V + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    return c / c[-1]


def _ranks(rng, cdf, n, chunk=1 << 24):
    out = np.empty(n, np.int32)
    for i in range(0, n, chunk):
        m = min(chunk, n - i)
        out[i:i + m] = np.searchsorted(cdf, rng.random(m), side="right")
    np.minimum(out, cdf.size - 1, out=out)
    return out


def tokens_to_csr(tok, V):
    """(D, L) int32 term ids → CsrMatrix of per-row unique ids and counts."""
    D, L = tok.shape
    srt = np.sort(tok, axis=1)
    head = np.ones((D, L), bool)
    head[:, 1:] = srt[:, 1:] != srt[:, :-1]
    pos = np.flatnonzero(head.ravel())
    counts = np.diff(np.append(pos, D * L)).astype(np.float64)
    indices = srt.ravel()[pos].astype(np.int32)
    indptr = np.zeros(D + 1, np.int64)
    np.cumsum(head.sum(axis=1), out=indptr[1:])
    return CsrMatrix(indptr, indices, counts, V)


def zipf_corpus(D, L, V, s=1.0, seed=20261015, chunk_docs=1 << 17):
    rng = np.random.default_rng(seed)
    cdf = _zipf_cdf(V, s)
    perm = rng.permutation(V).astype(np.int32)
    parts = []
    for d0 in range(0, D, chunk_docs):
        m = min(chunk_docs, D - d0)
        tok = perm[_ranks(rng, cdf, m * L)].reshape(m, L)
        parts.append(tokens_to_csr(tok, V))
    return concat_rows(parts, V)


def zipf_lda_corpus(D, L, V, k, s=1.0, alpha0=0.1, seed=20261015, chunk_docs=1 << 16):
    rng = np.random.default_rng(seed)
    cdf = _zipf_cdf(V, s)
    perms = np.stack([rng.permutation(V).astype(np.int32) for _ in range(k)])
    parts = []
    for d0 in range(0, D, chunk_docs):
        m = min(chunk_docs, D - d0)
        theta = rng.dirichlet(np.full(k, alpha0), size=m)
        cum = np.cumsum(theta, axis=1)
        cum[:, -1] = 1.0
        cum += np.arange(m)[:, None]
        u = rng.random((m, L)) + np.arange(m)[:, None]
        z = np.searchsorted(cum.ravel(), u.ravel(), side="right").reshape(m, L)
        z -= (np.arange(m) * k)[:, None]
        np.clip(z, 0, k - 1, out=z)
        tok = perms[z, _ranks(rng, cdf, m * L).reshape(m, L)]
        parts.append(tokens_to_csr(tok, V))
    return concat_rows(parts, V)


def concat_rows(parts, V):
    if len(parts) == 1:
        return parts[0]
    nnz = np.cumsum([0] + [p.nnz for p in parts])
    indptr = np.concatenate([parts[0].indptr[:1]] + [p.indptr[1:] + o for p, o in zip(parts, nnz[:-1])])
    return CsrMatrix(indptr, np.concatenate([p.indices for p in parts]),
                     np.concatenate([p.values for p in parts]), V)


def make_corpus(kind, D, L, V, k, seed):
    if kind == "zipf":
        return zipf_corpus(D, L, V, seed=seed)
    if kind == "zipf-lda":
        return zipf_lda_corpus(D, L, V, k, seed=seed)
    raise ValueError(f"unknown corpus kind {kind}")
