"""The fp64 E-step's per-document fixed cost, without in-kernel stamps: E-step time per minibatch at
capped inner-iteration counts (maxInnerIter = 1, 2, 4, 8, uncapped) over the same corpus and model
state, fitted as ms = fixed + per_iter · mean_iters.  The fixed part is everything a document pays
once — the worker loads, γ₀, the B block gather, the outputs — and the launch tail.

    python tools/iter_sweep.py [--corpus zipf-lda|zipf]
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
    p.add_argument("--corpus", default="zipf-lda", choices=["zipf", "zipf-lda"])
    p.add_argument("--burn", type=int, default=20)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--caps", default="1,2,4,8,0")
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    a = p.parse_args()
    import stc
    from stc import synth

    ctx = stc.Context(0)
    corpus = synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, a.seed)
    dc = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64 if a.dtype == "f64" else stc.STC_F32)
    # the model state: planted topics, or 20 uncapped minibatches from λ₀
    h0 = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                       seed=a.seed, dtype=a.dtype)
    h0.set_corpus(dc, a.docs)
    if a.corpus == "zipf-lda":
        h0.set_topics(synth.planted_topics(a.vocab, a.k, seed=a.seed))
    else:
        h0.init_random(a.seed)
        for _ in range(a.burn):
            h0.next(stats=False)
    lam = h0.topics()
    h0.close()
    rows = []
    for cap in [int(c) for c in a.caps.split(",")]:
        h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                          seed=a.seed, dtype=a.dtype, max_inner_iter=cap)
        h.set_corpus(dc, a.docs)
        h.set_topics(lam)
        h.next(stats=False)  # warm-up
        ctx.synchronize()
        c0 = h.counters()
        h.enable_timing(True)
        for _ in range(a.steps):
            h.next(stats=False)
        ctx.synchronize()
        ph = h.phase_times()
        c1 = h.counters()
        docs = c1["docs"] - c0["docs"]
        it = (c1["inner_iters"] - c0["inner_iters"]) / max(1, docs)
        rows.append({"max_inner_iter": cap, "mean_inner_iters": round(it, 3),
                     "estep_ms": round(ph["estep"], 4), "docs_per_minibatch": docs / a.steps})
        print(json.dumps(rows[-1]), flush=True)
        h.close()
    x = np.array([r["mean_inner_iters"] for r in rows])
    y = np.array([r["estep_ms"] for r in rows])
    b, c = np.polyfit(x, y, 1)
    print(json.dumps({"corpus": a.corpus, "dtype": a.dtype, "fit": {"fixed_ms": round(float(c), 4), "ms_per_iter": round(float(b), 4)},
                      "rows": rows}))


if __name__ == "__main__":
    main()
