"""A/B parity of two builds of libstc: the same E-step + a few next() steps, outputs compared bit for bit.

    python tools/ab_bitwise.py LIB_A LIB_B [--docs N] [--k K] [--dtype f64] [--env-a VAR=VAL] [--env-b VAR=VAL]

Each library runs in its own child process (STC_LIB selects it); the child writes γ, stat, the iteration
counts and λ after three next() steps to an .npz, and the parent compares the arrays with array_equal.
Used to show a kernel variant (a build-time switch) leaves every output unchanged before timing it.
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, docs, k, dtype):
    sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))
    import stc
    from stc import synth

    ctx = stc.Context.get(0)
    V = 1 << 18
    corpus = synth.zipf_corpus(docs, 200, V, seed=7)
    # a few longer rows: R = 6 (the LDS row set) and the 7-8-set launch
    rng = np.random.default_rng(3)
    lam = rng.gamma(100.0, 0.01, size=(V, k))
    g0 = rng.gamma(100.0, 0.01, size=(docs, k))
    h = stc.LdaHandle(ctx, k, V, dtype=dtype, mini_batch_fraction=0.05, seed=5)
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F32 if dtype == "f32" else stc.STC_F64)
    h.set_corpus(d, docs)
    h.set_topics(lam)
    gamma, stat, iters = h.estep(np.arange(docs), g0, want_stat=True)
    for _ in range(3):
        h.next(stats=False)
    np.savez(out, gamma=gamma, stat=stat, iters=iters, lam=h.topics(), alpha=h.alpha())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs=2)
    p.add_argument("--docs", type=int, default=20000)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--dtype", default="f64")
    p.add_argument("--child", default=None)
    p.add_argument("--env-a", action="append", default=[], help="VAR=VAL set for the first run only")
    p.add_argument("--env-b", action="append", default=[], help="VAR=VAL set for the second run only")
    a = p.parse_args()
    if a.child:
        child(a.child, a.docs, a.k, a.dtype)
        return
    outs = []
    with tempfile.TemporaryDirectory() as td:
        for i, lib in enumerate(a.libs):
            out = os.path.join(td, f"{i}.npz")
            env = dict(os.environ, STC_LIB=os.path.abspath(lib))
            env.update(kv.split("=", 1) for kv in (a.env_a if i == 0 else a.env_b))
            subprocess.run([sys.executable, __file__, *a.libs, "--docs", str(a.docs), "--k", str(a.k), "--dtype",
                            a.dtype, "--child", out], env=env, check=True)
            outs.append(dict(np.load(out)))
    ok = True
    for key in outs[0]:
        same = np.array_equal(outs[0][key], outs[1][key])
        ok &= same
        print(f"{key}: {'bitwise equal' if same else 'DIFFERENT'}"
              + ("" if same else f" (max abs diff {np.max(np.abs(outs[0][key] - outs[1][key])):.3e})"))
    print(f"mean iters {outs[0]['iters'].mean():.2f}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
