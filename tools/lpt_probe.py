"""How much of the headline E-step is its tail: the same minibatch E-step timed in sampling order and in
descending order of each document's (known, from a first run) iteration count — the longest-processing-
time-first bound on what any slot ordering could gain.

    python tools/lpt_probe.py [--docs 1000000] [--burn 20] [--reps 5]
    rocprofv3 --kernel-trace --output-format csv -d DIR -o lpt -- python3 tools/lpt_probe.py
    python tools/lpt_probe.py --trace DIR   (the E-step kernel's durations per ordering)

The wall times include the host copies of γ; under rocprofv3 the last 3·reps E-step launches are the
sampling-order, longest-first and random-order runs, in that order.

Warm state as bench.py's headline (configs[1]: 1M x 200 Zipf, V = 2^18, k = 100, fp64, 20 minibatches from
λ₀); then one Bernoulli(0.05) draw of members, γ₀ ~ Gamma(100, 1/100), E-step only (no sstats copy).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--burn", type=int, default=20)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--trace", default=None)
    p.add_argument("--workers", type=int, default=16)  # 1 under rocprofv3 (forked workers inherit the profiler)
    a = p.parse_args()
    if a.trace:
        import csv
        import glob

        f = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)[0]
        rows = [r for r in csv.DictReader(open(f)) if "k_estep_rows64_pers" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows[-3 * a.reps:]]
        out = {n: ms[i * a.reps:(i + 1) * a.reps] for i, n in enumerate(["sampling", "longest_first", "random"])}
        med = {n: float(np.median(v)) for n, v in out.items()}
        print(json.dumps({"kernel_ms": out, "median_ms": med, "gain": 1 - med["longest_first"] / med["sampling"]}))
        return
    import stc
    from stc import synth

    V = 1 << 18
    log = lambda m: print(f"[lpt] {m}", file=sys.stderr, flush=True)  # noqa: E731 (progress under a profiler)
    corpus = synth.zipf_corpus(a.docs, 200, V, workers=a.workers)
    log("corpus generated")
    ctx = stc.Context.get(0)
    h = stc.LdaHandle(ctx, a.k, V, dtype="f64", mini_batch_fraction=0.05, optimize_doc_concentration=True, seed=20261015)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h.set_corpus(d, a.docs)
    h.init_random(20261015)  # bench.py's seed: its warm state (≈ 155 iterations per document)
    for i in range(a.burn):
        h.next(stats=False)
        log(f"minibatch {i + 1}")
    rng = np.random.default_rng(5)
    ids = np.flatnonzero(rng.random(a.docs) < 0.05)
    g0 = rng.gamma(100.0, 0.01, size=(ids.size, a.k))

    def timed(ii, gg):
        best, out = [], None
        for _ in range(a.reps):
            ctx.synchronize()
            t0 = time.perf_counter()
            out = h.estep(ii, gg)
            best.append(time.perf_counter() - t0)
        log("timed")
        return out, float(np.median(best)) * 1e3

    (gam, _, it), t_samp = timed(ids, g0)
    order = np.argsort(-it, kind="stable")
    (gam2, _, it2), t_lpt = timed(ids[order], g0[order])
    perm = rng.permutation(ids.size)
    (_, _, _), t_rand = timed(ids[perm], g0[perm])
    same = bool(np.array_equal(gam2, gam[order]) and np.array_equal(it2, it[order]))
    print(json.dumps({"docs": int(ids.size), "mean_iters": float(it.mean()), "max_iters": int(it.max()),
                      "ms_sampling_order": t_samp, "ms_longest_first": t_lpt, "ms_random_order": t_rand,
                      "gain": 1 - t_lpt / t_samp, "gamma_bitwise_same": same}))


if __name__ == "__main__":
    main()
