"""Shared test inputs (seeded, small enough for the oracle to finish in seconds)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_npz(name):
    return np.load(os.path.join(GOLDEN, name))


def golden_json(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


def random_corpus(rng, D, V, min_nnz=1, max_nnz=40, max_count=6, empty_every=0):
    """Rows with sorted unique term ids and integer counts (Spark SparseVector semantics)."""
    import stc

    rows = []
    for d in range(D):
        if empty_every and d % empty_every == empty_every - 1:
            rows.append((np.zeros(0, np.int32), np.zeros(0)))
            continue
        n = int(rng.integers(min_nnz, max_nnz + 1))
        ids = np.sort(rng.choice(V, size=min(n, V), replace=False)).astype(np.int32)
        rows.append((ids, rng.integers(1, max_count + 1, ids.size).astype(np.float64)))
    return stc.CsrMatrix.from_rows(rows, V)


def long_run_corpus(rng, D, V, hot):
    """Every document holds the `hot` terms (the first in all documents, the others in most), plus 3-6
    random ones: the term-sorted entries have runs of thousands of entries — hundreds of sstats chunks,
    several full 32-chunk tiles (lda.hip k_fixup_tiles) — starting at odd offsets."""
    import stc

    hot = np.asarray(hot, np.int32)
    keep = rng.random((D, hot.size)) < np.linspace(1.0, 0.55, hot.size)
    cold = [np.setdiff1d(rng.choice(V, size=int(rng.integers(3, 7)), replace=False), hot) for _ in range(D)]
    rows = []
    for d in range(D):
        ids = np.unique(np.concatenate([hot[keep[d]], cold[d]])).astype(np.int32)
        rows.append((ids, rng.integers(1, 5, ids.size).astype(np.float64)))
    return stc.CsrMatrix.from_rows(rows, V)


def planted_corpus(rng, D, V, k, L=60, alpha=0.1):
    """A small LDA-generative corpus (topics = Zipf over their own term permutation)."""
    import stc

    ranks = np.arange(1, V + 1, dtype=np.float64)
    zipf = 1.0 / ranks
    zipf /= zipf.sum()
    topics = np.stack([zipf[np.argsort(rng.permutation(V))] for _ in range(k)])
    rows = []
    for _ in range(D):
        theta = rng.dirichlet(np.full(k, alpha))
        z = rng.choice(k, size=L, p=theta)
        terms = np.array([rng.choice(V, p=topics[t]) for t in z])
        u, c = np.unique(terms, return_counts=True)
        rows.append((u.astype(np.int32), c.astype(np.float64)))
    return stc.CsrMatrix.from_rows(rows, V), topics


def random_tokens(rng, n_docs, max_len=30, vocab=None):
    """Token lists covering every UTF-8 tail length 0–3 and multi-byte characters."""
    alphabet = list("abcdefghijklmnopqrstuvwxyz") + ["é", "ß", "ж", "中", "🙂", "Ω", "ü"]
    if vocab is None:
        vocab = ["".join(rng.choice(alphabet, size=int(rng.integers(1, 13)))) for _ in range(400)]
        vocab += ["", "a", "ab", "abc", "abcd", "the", "Holm", "Watson"]
    p = 1.0 / np.arange(1, len(vocab) + 1)
    p /= p.sum()
    docs = []
    for _ in range(n_docs):
        n = int(rng.integers(0, max_len + 1))
        docs.append([vocab[i] for i in rng.choice(len(vocab), size=n, p=p)])
    return docs
