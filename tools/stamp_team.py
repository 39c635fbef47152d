"""Where the team E-step spends its cycles: per-phase s_memtime stamps of lda_wide.hip k_estep_wide_mc
(--kernel mc, with STC_WIDE_TEAM=P), k_estep_wide_tc (--kernel tc: config 5's, --k 2000 --tokens 50
--vocab 262144) or lda_team64.hip k_estep_tgrid64 (--kernel tgrid, the fp64 default).

    make -C spark-text-clustering_amd/csrc stamp
    STC_LIB=spark-text-clustering_amd/stc/libstc_stamp.so python tools/stamp_team.py [--dtype f64 ...]

A config-4-shaped workload (k = 500, V = 2^20, 500 tokens per doc) on a smaller corpus; prints each
phase's share of the summed wave cycles and cycles per wave per inner iteration (8 waves per block,
P blocks per document).  The stamps fence the schedule: read SHARES, not absolute time.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))

PHASES = {"mc": ["per-doc preamble + block loads", "A: phi rows + reduce", "barriers, r, sum r*phi", "B: s partial",
                 "exchange: publish + wait + sums", "gamma, psi/exp", "outputs"],
          "tgrid": ["block loads", "A: phi FMAs + worker sums", "exchange: publish + poll + sums", "r, eps ballot, r reads",
                    "B: s FMAs + stores", "barrier 1", "psi phase (psi waves)", "barrier 2 (psi waves)",
                    "psi phase (others: empty)", "barrier 2 (others)"],
          "tc": ["per-doc preamble", "block loads + first eth", "A: phi partials + barrier 1",
                 "exchange: publish + poll + sums", "r, sum r*phi, barrier 2", "B: s + gamma/psi/exp",
                 "outputs + final exchange"]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=100_000)
    p.add_argument("--tokens", type=int, default=500)
    p.add_argument("--vocab", type=int, default=1 << 20)
    p.add_argument("--k", type=int, default=500)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--dtype", default="f64")
    p.add_argument("--burn", type=int, default=5)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--kernel", default="tgrid", choices=sorted(PHASES))
    a = p.parse_args()
    phases = PHASES[a.kernel]
    assert "stamp" in os.environ.get("STC_LIB", ""), "set STC_LIB to the stamp build"
    import stc
    from stc import synth

    corpus = synth.make_corpus("zipf", a.docs, a.tokens, a.vocab, a.k, a.seed, workers=8)
    print("corpus generated", file=sys.stderr, flush=True)
    ctx = stc.Context(0)
    lib = stc._lib.load()
    reader = lib.stc_debug_stamps_team64 if a.kernel == "tgrid" else lib.stc_debug_stamps_wide
    reader.restype = C.c_int
    reader.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    buf = (C.c_ulonglong * 12)()
    dc = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if a.dtype == "f32" else stc.STC_F64)
    h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                      seed=a.seed, dtype=a.dtype)
    h.set_corpus(dc, a.docs)
    h.init_random(a.seed)
    for i in range(a.burn):
        h.next(stats=False)
        ctx.synchronize()
        print(f"burn-in minibatch {i + 1}", file=sys.stderr, flush=True)
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
    tot = cyc[:len(phases)].sum()
    P = int(os.environ.get("STC_WIDE_TEAM", "0")) or {"tgrid": -(-a.k // 104), "tc": -(-a.k // 1024)}.get(a.kernel)
    out = {"k": a.k, "dtype": a.dtype, "team": P or "auto", "docs": int(docs),
           "mean_inner_iters": iters / max(1, docs), "share": {}, "cycles_per_block_wave_iter": {}}
    waves = 8 * (P or 1)
    for i, name in enumerate(phases):
        out["share"][name] = round(cyc[i] / tot, 4)
        out["cycles_per_block_wave_iter"][name] = round(cyc[i] / (waves * max(1, iters)), 1)
    out["note"] = "per-iteration cycles assume `team` blocks per document (set STC_WIDE_TEAM)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
