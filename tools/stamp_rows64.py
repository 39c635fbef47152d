"""Where an iteration of the fp64 rows-split E-step (lda_rows64.hip) spends its cycles: per-phase
s_memtime stamps from the diagnostic build.

    make -C spark-text-clustering_amd/csrc stamp          # → stc/libstc_stamp.so (never the product)
    STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_rows64.py [--corpus zipf-lda]

Runs bench.py's corpus and model state (20 burn-in minibatches, then --steps measured ones) and prints
each phase's cycles per wave per inner iteration.  The stamps fence the schedule (an lgkmcnt(0) drain at
each), so read the split, not absolute time (cdna_hip_programming.md §7, In-kernel stamps).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))

PHASES = ["init: loads, gamma0, first eth", "A: eth reads + phi FMAs + all-reduce", "r, eps ballot, sum|dgamma|",
          "B: s FMAs + stores", "barrier 1", "psi phase (psi waves)", "barrier 2 (psi waves)", "outputs",
          "psi phase (other waves)", "barrier 2 (other waves)", "prologue: worker loads, gamma0, first eth"]
PER_DOC = (0, 7, 10)  # once per document: block loads, outputs, prologue


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--tokens", type=int, default=200)
    p.add_argument("--vocab", type=int, default=1 << 18)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--corpus", default="zipf", choices=["zipf", "zipf-lda"])
    p.add_argument("--burn", type=int, default=20)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--seed", type=int, default=20261015)
    a = p.parse_args()
    assert "stamp" in os.environ.get("STC_LIB", ""), "set STC_LIB to the stamp build"
    import stc
    from stc import synth

    ctx = stc.Context(0)
    lib = stc._lib.load()
    reader = lib.stc_debug_stamps_rows64
    reader.restype = C.c_int
    reader.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    n = len(PHASES)
    buf = (C.c_ulonglong * 12)()
    corpus = synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, a.seed)
    dc = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                      seed=a.seed, dtype="f64")
    h.set_corpus(dc, a.docs)
    if a.corpus == "zipf-lda":
        h.set_topics(synth.planted_topics(a.vocab, a.k, seed=a.seed))
    else:
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
    cyc = np.array(buf[:n], dtype=np.float64)
    docs = c1["docs"] - c0["docs"]
    iters = c1["inner_iters"] - c0["inner_iters"]
    W = 4
    out = {"k": a.k, "corpus": a.corpus, "docs": int(docs), "mean_inner_iters": iters / max(1, docs),
           "cycles_per_wave_iter": {}}
    for i, name in enumerate(PHASES):
        out["cycles_per_wave_iter"][name] = round(cyc[i] / (W * max(1, iters)), 1)
    out["cycles_per_wave_iter"]["total"] = round(cyc.sum() / (W * max(1, iters)), 1)
    out["cycles_per_wave_doc"] = {PHASES[i]: round(cyc[i] / (W * max(1, docs)), 1) for i in PER_DOC}
    out["cycles_per_wave_doc"]["loop"] = round(sum(cyc[i] for i in range(n) if i not in PER_DOC) / (W * max(1, docs)), 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
