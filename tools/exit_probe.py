"""Reproduce and locate the exit-time SIGSEGV of processes that ran the team E-step under rocprofv3
(VERDICT r2 #3): a small k = 2000 fp64 model forced onto the cooperative team kernel, three next()
calls, then exit.  /proc/self/maps is written to OUT at interpreter exit, so the raw addresses of a
crash stack can be mapped to (library, offset) afterwards (tools/symbolize_stack.py).

    rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/exit_probe.py OUT [--close]

--close releases every native object (LDA handle, device CSR, context) before the interpreter exits.
"""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    out = sys.argv[1]
    close = "--close" in sys.argv
    os.environ.setdefault("STC_WIDE_TEAM", "2")
    import numpy as np

    import stc
    from helpers import random_corpus

    atexit.register(lambda: open(out, "w").write(open("/proc/self/maps").read()))
    rng = np.random.default_rng(5)
    corpus = random_corpus(rng, 2000, 4096, 1, 60)
    ctx = stc.Context(0)
    h = stc.LdaHandle(ctx, 2000, corpus.num_cols, mini_batch_fraction=0.2, seed=3, dtype="f64")
    d = stc.DeviceCsr.upload(ctx, corpus, stc.STC_F64)
    h.set_corpus(d, corpus.num_rows)
    h.init_random(3)
    for _ in range(3):
        h.next(stats=False)
    ctx.synchronize()
    print("probe: 3 team steps done, close =", close, flush=True)
    if close:
        h.close()
        d.free()
        ctx.close()


if __name__ == "__main__":
    main()
