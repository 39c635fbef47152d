"""Where an E-step inner iteration spends its cycles: per-phase s_memtime stamps (diagnostic build).

    make -C spark-text-clustering_amd/csrc stamp          # → stc/libstc_stamp.so (never the product)
    STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_estep.py [--k 100 ...]

Runs the bench workload (bench.py's corpus and model state) for a few minibatches and prints each
phase's share of the summed wave cycles, and cycles per wave per inner iteration.  The stamps fence
the schedule, so read SHARES, not absolute time (cdna_hip_programming.md §7, In-kernel stamps).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))

PHASES = ["eps, partner barrier, init", "A: eth reads + phi FMAs", "phi exchange (LDS+barrier)", "r, sum r*dot",
          "psi(sum gamma')", "B: s FMAs", "reduce-scatter", "C: gamma, sum|dgamma|", "D: psi/exp, eth->LDS",
          "outputs", "loads: ids + staged B rows", "preamble: indptr, gamma0 sampling"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--tokens", type=int, default=200)
    p.add_argument("--vocab", type=int, default=1 << 18)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--burn", type=int, default=20)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--seed", type=int, default=20261015)
    a = p.parse_args()
    assert "stamp" in os.environ.get("STC_LIB", ""), "set STC_LIB to the stamp build"
    import stc
    from stc import synth

    ctx = stc.Context(0)
    lib = stc._lib.load()
    reader = lib.stc_debug_stamps_grid  # the fp32 grid kernel (lda_grid.hip)
    reader.restype = C.c_int
    reader.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    buf = (C.c_ulonglong * 12)()
    corpus = synth.make_corpus("zipf", a.docs, a.tokens, a.vocab, a.k, a.seed)
    dc = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32)
    h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                      seed=a.seed, dtype="f32")
    h.set_corpus(dc, a.docs)
    h.init_random(a.seed)
    for _ in range(a.burn):
        h.next(stats=False)
    ctx.synchronize()
    assert reader(buf, 12, 1) == 0
    c0 = h.counters()
    for _ in range(a.steps):
        h.next(stats=False)
    ctx.synchronize()
    assert reader(buf, 12, 1) == 0
    c1 = h.counters()
    cyc = np.array(buf[:], dtype=np.float64)
    docs = c1["docs"] - c0["docs"]
    iters = c1["inner_iters"] - c0["inner_iters"]
    tot = cyc.sum()
    # every wave stamps; waves per doc = 2 for k <= 104
    W = 2 if a.k <= 104 else 4
    out = {"k": a.k, "docs": int(docs), "mean_inner_iters": iters / max(1, docs), "waves_per_doc": W,
           "cycles_per_wave_iter": {}, "share": {}}
    for i, name in enumerate(PHASES):
        if cyc[i] == 0:
            continue
        out["share"][name] = round(cyc[i] / tot, 4)
        out["cycles_per_wave_iter"][name] = round(cyc[i] / (W * max(1, iters)), 1)
    out["cycles_per_wave_iter"]["total"] = round(tot / (W * max(1, iters)), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
