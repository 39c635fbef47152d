"""Tokenizer (K0) throughput probe: D docs × L bytes of seeded ASCII text (18 % separators, mixed
case) through stc_tokenize.  Kernel times come from rocprofv3 --kernel-trace --stats
(k_count / k_emit); this script prints the host wall time per call (PCIe included)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "spark-text-clustering_amd"))
import stc  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--docs", type=int, default=200_000)
p.add_argument("--bytes-per-doc", type=int, default=1200)
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
rng = np.random.default_rng(20261015)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ", np.uint8)
n = a.docs * a.bytes_per_doc
text = alpha[rng.integers(0, alpha.size, n)]
text[rng.random(n) < 0.18] = ord(" ")
off = np.arange(a.docs + 1, dtype=np.int64) * a.bytes_per_doc
ctx = stc.Context(0)
lib = ctx.lib
import ctypes as C  # noqa: E402
from stc import _lib as L  # noqa: E402
out = np.zeros(n + n // 2, np.uint8)  # stc_tokenize's bound: lower-casing may grow text by half
tok = np.zeros(n + a.docs + 1, np.int64)
doc = np.zeros(a.docs + 1, np.int64)
nb, nt = C.c_int64(), C.c_int64()
ts = []
for r in range(a.reps + 1):
    t0 = time.perf_counter()
    L.check(lib.stc_tokenize(ctx.handle, L.ptr(text, C.c_uint8), n, L.ptr(off, C.c_int64), a.docs,
                             L.ptr(out, C.c_uint8), out.size, C.byref(nb), L.ptr(tok, C.c_int64), C.byref(nt),
                             L.ptr(doc, C.c_int64)))
    ts.append(time.perf_counter() - t0)
print(json.dumps({"docs": a.docs, "bytes": n, "tokens": nt.value, "kept_bytes": nb.value,
                  "host_ms_per_call_incl_pcie": 1e3 * float(np.median(ts[1:]))}))
