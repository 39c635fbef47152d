"""Per-document E-step iteration counts at the bench's model state, and how far the fp32 E-step's γ moves
from the fp64 one as a function of that count (the input to the mixed mode's fp64 re-solve threshold,
DESIGN.md §4): λ after `--burn` fp64 minibatches from λ₀ (the bench's warm state), then one E-step over
`--sample` random documents in fp64 and in fp32 from the same λ and γ₀.

    python tools/iter_hist.py [--corpus zipf|zipf-lda] > gpurun_out/iter_hist.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--tokens", type=int, default=200)
    p.add_argument("--vocab", type=int, default=1 << 18)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--corpus", default="zipf", choices=["zipf", "zipf-lda"])
    p.add_argument("--burn", type=int, default=20)
    p.add_argument("--sample", type=int, default=50000)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--workers", type=int, default=16)
    a = p.parse_args()
    import stc
    from stc import synth

    corpus = synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, a.seed, 0, a.docs, a.workers)
    ctx = stc.Context(0)
    d64 = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                      seed=a.seed, dtype="f64")
    h.set_corpus(d64, a.docs)
    if a.corpus == "zipf-lda":
        h.set_topics(synth.planted_topics(a.vocab, a.k, seed=a.seed))
    else:
        h.init_random(a.seed)
    for i in range(a.burn):
        h.next(stats=False)
        print(f"burn {i + 1}", file=sys.stderr, flush=True)
    lam, alpha = h.topics(), h.alpha()
    rng = np.random.default_rng(1)
    ids = rng.choice(a.docs, size=a.sample, replace=False)
    g0 = rng.gamma(100.0, 0.01, size=(a.sample, a.k))
    g64, _, it64 = h.estep(ids, g0)
    d32 = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32)
    h32 = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                        seed=a.seed, dtype="f32")
    h32.set_corpus(d32, a.docs)
    h32.set_topics(lam)
    h32.set_alpha(alpha)
    g32, _, it32 = h32.estep(ids, g0)
    rel = np.max(np.abs(g32 - g64) / g64, axis=1)
    out = {"corpus": a.corpus, "docs": a.docs, "sample": a.sample, "burn": a.burn, "mean_iters_f64": float(it64.mean()),
           "max_iters_f64": int(it64.max()), "percentiles_f64": {q: float(np.percentile(it64, q)) for q in (50, 90, 99, 99.9)}}
    tot = float(it64.sum())
    out["above"] = {str(t): {"docs": float((it64 > t).mean()), "iteration_share": float(it64[it64 > t].sum() / tot),
                             "max_gamma_rel_f32_below": float(rel[it64 <= t].max()) if np.any(it64 <= t) else None}
                    for t in (100, 200, 300, 500, 1000, 2000)}
    edges = [0, 50, 100, 200, 300, 500, 1000, 2000, 10 ** 9]
    out["gamma_rel_f32_by_iters"] = [
        {"iters": f"({lo}, {hi}]", "docs": int(((it64 > lo) & (it64 <= hi)).sum()),
         "median": float(np.median(rel[(it64 > lo) & (it64 <= hi)])) if np.any((it64 > lo) & (it64 <= hi)) else None,
         "max": float(rel[(it64 > lo) & (it64 <= hi)].max()) if np.any((it64 > lo) & (it64 <= hi)) else None}
        for lo, hi in zip(edges[:-1], edges[1:])]
    out["iters_equal_f32_f64"] = float((it32 == it64).mean())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
