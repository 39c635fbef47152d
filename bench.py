"""Benchmark: online-LDA minibatch steps (E-step + sstats + [RCCL all-reduce] + M-step) on MI355X.

Workload (BASELINE.json configs[1]): a synthetic Zipfian corpus of 1M docs × 200 tokens, V = 2^18,
online LDA k = 100, subsamplingRate 0.05 (≈50k docs per minibatch).  A "step" is one
OnlineLDAOptimizer.next(): device-side membership sampling, the E-step over the minibatch, the
term-sorted sufficient statistics, the all-reduce (N > 1) and the λ / expElogβ / α update.  The
corpus is resident in HBM before the timed region.  The headline computes in fp64 like Spark's
Breeze Double E-step (--dtype f64); the fp32 path and the planted-topic (warm) model state are
reported as secondary lines ("secondary") in the same JSON object at N = 1.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype f64|f32] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N   (one rank per GPU)

Multi-GPU (configs[2]: "the same 1M-doc corpus sharded at 2/4/8 GPUs"): --scaling strong (default)
gives rank r the rows [r·D/N, (r+1)·D/N) of ONE corpus (corpusSize = D); --scaling weak gives every
rank its own D-doc corpus (corpusSize = N·D).  One RCCL all-reduce of the k×V sstats per step.

Rank 0 prints ONE JSON line.  value = Σ_ranks minibatch docs in the K timed steps ÷ the
max-over-ranks wall time.  Model state: timing starts after exactly
--state-minibatches (20) minibatches from λ₀ (burn-in + warmup), so the inner-iteration count does
not depend on --warmup; the first 3 minibatches from λ₀ are timed separately as the "cold" figure.
roofline: the dominant kernel (the training E-step: k_estep_rows64 for fp64, k_estep_grid for
fp32; one launch per minibatch): SURVEY.md §8(d) algorithmic bytes per doc
(nnz·(4 + s) + 2·nnz·k·s + s·k, s = 8 for fp64, 4 for fp32) × the launch's docs ÷ its HIP-event time
on the library stream; traffic: the PMC FETCH_SIZE(×2, gfx950) + WRITE_SIZE per launch of that
kernel from the committed rocprofv3 summary of this workload (profiles/, tools/gpu.sh prof).
roofline_compute: the same kernel's flops (4·nnz·k per inner iteration) against the dtype's peak.
cpu_baseline: oracle/lda_oracle.c oracle_minibatch — one full submitMiniBatch + updateLambda +
updateAlpha in Spark's structure (fp64, per-thread dense k×V stats, OpenMP on the host cores) —
timed on whole minibatches of the same corpus at the GPU model's state after the timed steps.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
PEAK_TFS = {"f32": 157.3, "f64": 78.6, "mixed": 157.3}  # MI355X dense vector peaks (fp32 = MFMA f32 rate; fp64
# vector); mixed runs the fp32 E-step (its fp64 re-solve of the slow documents is a few % of the iterations)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_traffic.json")
METRIC = "LDA E-step docs/sec (node) at k=100, V=2^18; % of HBM roofline"  # the configs[1] metric


# BASELINE.json configs: 2 (the headline), 4 (its per-GPU shard: 10M docs over 8 GPUs), 5
PRESETS = {2: dict(docs=1_000_000, tokens=200, vocab=1 << 18, k=100),
           4: dict(docs=1_250_000, tokens=500, vocab=1 << 20, k=500),
           5: dict(docs=1_000_000, tokens=50, vocab=1 << 18, k=2000)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, default=2, choices=sorted(PRESETS),
                   help="BASELINE.json configs[n-1] shape preset (docs/tokens/vocab/k); explicit flags override")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--docs", type=int, default=None, help="documents of the corpus (per GPU if weak)")
    p.add_argument("--tokens", type=int, default=None)
    p.add_argument("--vocab", type=int, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--corpus", default="zipf", choices=["zipf", "zipf-lda"])
    p.add_argument("--state", default="burn-in", choices=["burn-in", "planted"],
                   help="model state of the timed steps: after --state-minibatches from λ₀, or (zipf-lda) "
                        "the planted topicsMatrix that generated the corpus (SURVEY §8(d) state B)")
    p.add_argument("--dtype", default="f64", choices=["f32", "f64", "mixed"])
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--state-minibatches", type=int, default=20,
                   help="minibatches applied from λ₀ before timing (burn-in + warmup)")
    p.add_argument("--workers", type=int, default=16, help="corpus-generation processes (before GPU init)")
    p.add_argument("--no-secondary", action="store_true", help="headline only (no fp32 / planted / featurisation)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--featurisation-only", action="store_true",
                   help="only the HashingTF -> IDF line (for profiling its kernels)")
    p.add_argument("--no-hbm-copy", action="store_true", help="skip the device-copy HBM probe")
    p.add_argument("--launch", default="auto", choices=["auto", "group"],
                   help="group: drive the GPUs through one stc_group even at N = 1 (with STC_GROUP_RCCL=1 "
                        "its RCCL communicator, ncclCommInitAll, and one host thread per member)")
    a = p.parse_args()
    for key, v in PRESETS[a.config].items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    return a


def bytes_per_doc(nnz, k, s):
    """ids + counts (4 + s B per nnz), one k-wide row gathered and one scattered per
    nnz, γ out (s·k B per doc); s = value size (8 fp64, 4 fp32)."""
    return nnz * (4.0 + s), 2.0 * nnz * k * s, s * k


def algorithmic_bytes(nnz, k, docs, dtype):
    s = 8.0 if dtype == "f64" else 4.0  # (mixed: the fp32 data path)
    a, b, c = bytes_per_doc(nnz, k, s)
    return a + b + docs * c


# the E-step kernels' sources: a PMC entry counts only if it was measured on these exact files
ESTEP_SOURCES = ("lda_rows64.hip", "psi64.h", "lda_grid.hip", "lda_wide.hip", "lda_team64.hip", "team_exchange.h", "lda.hip",
                 "estep_common.h", "lda_kernels.h")


def estep_sources_sha():
    import hashlib

    h = hashlib.sha256()
    for f in ESTEP_SOURCES:
        with open(os.path.join(ROOT, "spark-text-clustering_amd", "csrc", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


# the featurisation kernels' sources: its PMC entry counts only if measured on these exact files
FEAT_SOURCES = ("hashing_tf.hip", "idf.hip", "stc_internal.h")
FEAT_PMC = os.path.join(ROOT, "profiles", "r06_featurisation_pmc.json")


def feat_sources_sha():
    import hashlib

    h = hashlib.sha256()
    for f in FEAT_SOURCES:
        with open(os.path.join(ROOT, "spark-text-clustering_amd", "csrc", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def feat_traffic():
    """HBM bytes per call of each featurisation stage from the committed PMC summary
    (tools/gpu.sh feat → tools/feat_pmc_summary.py), if measured on this tree's sources."""
    try:
        with open(FEAT_PMC) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, "no featurisation PMC summary committed"
    if pm.get("feat_sources_sha") != feat_sources_sha():
        return None, f"{os.path.basename(FEAT_PMC)} was measured on other featurisation sources"
    return {k: v["bytes_per_call"] for k, v in pm["stages"].items()}, f"{os.path.basename(FEAT_PMC)} ({pm.get('note', '')})"


def pmc_traffic(a, dtype, corpus):
    """HBM bytes per launch of the training E-step kernel from the committed PMC summary
    (tools/pmc_summary.py over tools/gpu.sh prof's separate FETCH_SIZE / WRITE_SIZE passes), if it
    was measured on this workload; FETCH_SIZE ×2 per the gfx950 correction (MI355X_MICROARCH.md)."""
    try:
        with open(PMC_SUMMARY) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary committed"
    want = (a.docs, a.k, a.vocab, a.tokens, a.fraction, corpus, dtype)
    for e in pm.get("entries", [pm]):
        w = e.get("workload", {})
        if (w.get("docs"), w.get("k"), w.get("vocab"), w.get("tokens"), w.get("fraction"), w.get("corpus"),
                w.get("dtype", "f32")) != want:
            continue
        b = e.get("estep_kernel_bytes_per_launch")
        if not e.get("estep_kernel") or not b:
            return None, f"PMC entry {e.get('tag', '?')} names no E-step kernel (broken summary)"
        sha = estep_sources_sha()
        if e.get("estep_sources_sha") != sha:
            return None, (f"PMC entry {e.get('tag', '?')} was measured on other E-step sources "
                          f"({e.get('estep_sources_sha')} vs HEAD {sha}): not a measurement of this code")
        # the K6 window's bytes (E-step kernel + the sstats phase: sort, SpMM, stat clear) when the summary
        # has them (round 5+), else the whole E-step phase per minibatch
        return {"kernel": b, "window": e.get("k6_window_bytes_per_step") or e.get("estep_phase_bytes_per_step")}, \
            f"{os.path.basename(PMC_SUMMARY)} ({e.get('note', '')})"
    return None, "no PMC summary committed for this workload"


def hbm_copy_gbs(device):
    """STREAM-style device-to-device copy (1 GiB, hipMemcpy through libamdhip64 via ctypes, timed with
    HIP events) for the measured-HBM figure next to the 8 TB/s spec.  Reported, never fatal."""
    import ctypes as C

    try:
        hip = C.CDLL("libamdhip64.so.7")  # the runtime libstc.so links (torch/lib carries its own copy)
        n = 1 << 30
        a, b = C.c_void_p(), C.c_void_p()
        e0, e1 = C.c_void_p(), C.c_void_p()
        hip.hipGetErrorString.restype = C.c_char_p
        for what, rc in (("hipSetDevice", lambda: hip.hipSetDevice(C.c_int(int(device)))),
                         ("hipMalloc", lambda: hip.hipMalloc(C.byref(a), C.c_size_t(n))),
                         ("hipMalloc", lambda: hip.hipMalloc(C.byref(b), C.c_size_t(n)))):
            r = rc()
            if r != 0:
                return f"{what} failed: {r} {hip.hipGetErrorString(r).decode()}"
        hip.hipMemset(a, 1, C.c_size_t(n))
        hip.hipEventCreate(C.byref(e0))
        hip.hipEventCreate(C.byref(e1))
        for _ in range(3):
            hip.hipMemcpy(b, a, C.c_size_t(n), 3)  # hipMemcpyDeviceToDevice
        hip.hipDeviceSynchronize()
        reps = 10
        hip.hipEventRecord(e0, None)
        for _ in range(reps):
            hip.hipMemcpyAsync(b, a, C.c_size_t(n), 3, None)
        hip.hipEventRecord(e1, None)
        hip.hipEventSynchronize(e1)
        ms = C.c_float()
        hip.hipEventElapsedTime(C.byref(ms), e0, e1)
        hip.hipFree(a)
        hip.hipFree(b)
        return 2.0 * n * reps / (ms.value * 1e-3) / 1e9 if ms.value > 0 else "no timing"
    except Exception as e:
        return f"copy probe failed: {type(e).__name__}: {e}"[:200]


def cpu_baseline(h, corpus, a, budget_s=12.0):
    """oracle/lda_oracle.c oracle_minibatch: whole submitMiniBatch + updateLambda + updateAlpha steps
    (fp64, Spark's structure: per-thread dense k×V stats summed like treeReduce, OpenMP over the
    host cores) on Bernoulli(fraction) minibatches of the same corpus, starting from the GPU model
    after the timed steps.  Only the oracle call is timed (membership and γ₀ generation are not)."""
    from oracle import c_oracle

    if not c_oracle.available():
        return None
    # the host cores this process may use: the lease's share (OMP_NUM_THREADS, which the GPU box sets to
    # its 16-core share per GPU), else every core in the affinity mask
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = omp or len(os.sched_getaffinity(0))
    why = "OMP_NUM_THREADS (the lease's core share)" if omp else "the process's affinity mask"
    lam = np.ascontiguousarray(h.topics().T)  # k×V, Spark's internal orientation
    alpha = np.ascontiguousarray(h.alpha())
    eta = h.eta()
    rng = np.random.default_rng(a.seed + 1)
    D = corpus.num_rows
    batch_size = np.ceil(a.fraction * D)
    done = iters = steps = 0
    dt = 0.0
    while dt < budget_s and steps < 8:
        ids = np.flatnonzero(rng.random(D) < a.fraction)
        g0 = rng.gamma(100.0, 0.01, size=(ids.size, a.k))
        rho = (1024.0 + 21 + steps) ** -0.51
        t1 = time.perf_counter()
        tot = c_oracle.minibatch(corpus.indptr, corpus.indices, corpus.values, ids, g0, lam, alpha, eta, rho,
                                 D / batch_size, True, n_threads=threads)
        dt += time.perf_counter() - t1
        done += ids.size
        iters += max(tot, 0)
        steps += 1
    return {"value": done / dt, "unit": "docs/s", "cores": threads, "kind": "port",
            "sample": f"{steps} whole minibatch steps ({done} docs, Bernoulli({a.fraction}) of the same corpus; "
                      f"E-step + per-thread dense k×V stats + reduce + λ/α update, fp64) from the GPU model "
                      f"after the timed steps; oracle/lda_oracle.c oracle_minibatch, OpenMP {threads} threads = {why}; "
                      f"mean inner iters {iters / max(1, done):.1f}; {dt:.1f} s"}


def featurization(stc, ctx, a, log, tokens, reps=5):
    """HashingTF (2^18 buckets, Spark 2.4.3's murmur3 tail) → IDF(minDocFreq = 2) fit → TF·IDF transform
    with the reference's 1e-4 floor (LDAClustering.scala:154-192), all on the GPU over a token corpus
    already resident in HBM (stc_tokens_upload before timing).  One pass = the three calls, each
    synchronised; tokens/s over the mean of `reps` passes after one warm-up pass."""
    (blob, tok_off, doc_off), _ = tokens
    n_tok, n_docs = tok_off.size - 1, doc_off.size - 1
    dt = stc.DeviceTokens(ctx, blob, tok_off, doc_off)
    htf = stc.HashingTF(numFeatures=a.vocab, ctx=ctx)
    idf = stc.IDF(minDocFreq=2, ctx=ctx)

    def one():
        ctx.synchronize()
        t0 = time.perf_counter()
        d = htf.transform_tokens_device(dt, stc.STC_F64)
        ctx.synchronize()
        t1 = time.perf_counter()
        m = idf.fit_device(d)
        ctx.synchronize()
        t2 = time.perf_counter()
        m.transform_device(d, zero_floor=1e-4)
        ctx.synchronize()
        t3 = time.perf_counter()
        nnz = d.nnz
        d.free()
        return np.array([t1 - t0, t2 - t1, t3 - t2]), nnz

    one()
    ts, nnz = [], 0
    for _ in range(reps):
        t, nnz = one()
        ts.append(t)
    t = np.mean(ts, axis=0)
    dt.free()
    V = a.vocab
    # algorithmic bytes: HashingTF reads the blob + offsets once and writes the CSR; IDF fit reads the
    # CSR's indices and writes df + idf; the transform reads indices + idf[j] + values, writes values
    # (a resident upload keeps its token offsets as u32 when the blob is under 4 GiB: stc_tokens_upload)
    off_b = 4.0 if blob.size + 64 <= 1 << 32 else 8.0
    b_hash = blob.size + off_b * (n_tok + 1) + 8.0 * (n_docs + 1) + nnz * (4 + 8) + 8.0 * (n_docs + 1)
    b_fit = nnz * 4 + 2 * 8.0 * V  # a HashingTF matrix's values are known > 0: df reads the ids only
    b_tr = nnz * (4 + 8 + 8) + 8.0 * V
    total = float(t.sum())
    traffic, traffic_src = feat_traffic()
    return {
        "label": f"featurisation: HashingTF(2^{int(V).bit_length() - 1}, spark24 murmur3) -> IDF(2).fit -> "
                 "transform(1e-4 floor), tokens resident in HBM",
        "value": n_tok / total, "unit": "tokens/s", "dtype": "f64 (values), int32 (indices)",
        "corpus": f"{n_docs} docs x {n_tok // max(1, n_docs)} tokens, Zipf(1) over a seeded 2^18-word "
                  f"dictionary (1-12 chars, 1-4 byte UTF-8: every murmur3 tail length)",
        "tokens": n_tok, "utf8_bytes": int(blob.size), "nnz": int(nnz),
        "ms": {"hashing_tf": round(t[0] * 1e3, 3), "idf_fit": round(t[1] * 1e3, 3), "idf_transform": round(t[2] * 1e3, 3)},
        "roofline": {"bound": "hbm", "achieved": (b_hash + b_fit + b_tr) / total / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": (b_hash + b_fit + b_tr) / total / 1e9 / HBM_PEAK_GBS,
                     "algorithmic_bytes": {"hashing_tf": b_hash, "idf_fit": b_fit, "idf_transform": b_tr},
                     "traffic": traffic, "traffic_source": traffic_src},
    }


class _Single:
    """one stc_lda on this process's context (N = 1, or one rank per GPU under torchrun)"""

    def __init__(self, stc, ctx, a, dtype, dcorp, total):
        self.ctx = ctx
        self.h = stc.LdaHandle(ctx, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                               seed=a.seed, dtype=dtype)
        self.h.set_corpus(dcorp, total)

    def sync(self):
        self.ctx.synchronize()

    def counters(self):  # (this process's view, the local view)
        c = self.h.counters()
        return c, c

    def phases(self):
        return self.h.phase_times(), None


class _Group:
    """one stc_group over N devices from this process (stc_group_*: the JVM drop-in's local[*] form)"""

    def __init__(self, stc, a, dtype, corpus, devices):
        self.h = stc.LdaGroup(devices, a.k, a.vocab, mini_batch_fraction=a.fraction, optimize_doc_concentration=True,
                              seed=a.seed, dtype=dtype)
        self.h.set_corpus(corpus)

    def sync(self):
        self.h.synchronize()

    def counters(self):  # (Σ over the members, member 0)
        cs = self.h.counters()
        tot = {key: sum(c[key] for c in cs) for key in cs[0] if key != "kernels"}
        tot["kernels"] = {f: sum(c["kernels"][f] for c in cs) for f in cs[0]["kernels"]}
        return tot, cs[0]

    def phases(self):  # member 0's phase times, and the slowest member's E-step
        ps = self.h.phase_times()
        return ps[0], max(p["estep"] for p in ps)


def run_state(m, lam0, barrier, log, a, dtype, steps, warmup):
    """One training run on model m (_Single / _Group): λ₀ (random Gamma, or the given topicsMatrix), 3
    timed cold minibatches, burn-in + warmup to the fixed state, then exactly `steps` timed minibatches."""
    h = m.h
    if lam0 is None:
        h.init_random(a.seed)
    else:
        h.set_topics(lam0)
    m.sync()
    cc0, _ = m.counters()
    t0 = time.perf_counter()
    n_cold = 3
    for _ in range(n_cold):
        h.next(stats=False)
    m.sync()
    cold_s = time.perf_counter() - t0
    cc1, _ = m.counters()
    cold = {"docs_per_s": (cc1["docs"] - cc0["docs"]) / cold_s,
            "mean_inner_iters": (cc1["inner_iters"] - cc0["inner_iters"]) / max(1, cc1["docs"] - cc0["docs"]),
            "minibatches": n_cold}
    burn = max(0, a.state_minibatches - n_cold - warmup)
    log(f"{burn + warmup} untimed minibatches ({dtype})")
    for i in range(burn + warmup):
        h.next(stats=False)
        if i % 4 == 3:  # progress (a profiler pass serialises kernels: keep the log moving)
            m.sync()
            log(f"  minibatch {n_cold + i + 1}")
    m.sync()
    c0, l0 = m.counters()
    h.enable_timing(True)
    barrier()
    log(f"timing {steps} steps ({dtype})")
    t_start = time.perf_counter()
    for _ in range(steps):
        h.next(stats=False)
    barrier()
    elapsed = time.perf_counter() - t_start
    phases, estep_max = m.phases()
    c1, l1 = m.counters()
    return {"elapsed": elapsed, "phases": phases, "estep_ms_slowest_member": estep_max, "cold": cold,
            "docs": c1["docs"] - c0["docs"], "entries": c1["entries"] - c0["entries"],
            "iters": c1["inner_iters"] - c0["inner_iters"], "cap_hits": c1["cap_hits"] - c0["cap_hits"],
            "docs_local": l1["docs"] - l0["docs"], "entries_local": l1["entries"] - l0["entries"],
            "iters_local": l1["inner_iters"] - l0["inner_iters"],
            # the E-step kernels the library actually launched in the timed steps (stc_lda_kernel_counts)
            "kernels": {f: l1["kernels"][f] - l0["kernels"][f] for f in l1["kernels"] if l1["kernels"][f] > l0["kernels"][f]}}


# north-star parity of each dtype (tests/test_gpu_config1.py: configs[0] against the oracle)
PARITY = {"f64": "north-star bars met: topicsMatrix 1e-9 (bar 1e-4), logPerplexity 1e-10 (bar 1e-5), identical "
                 "top-10 terms on configs[0] (tests/test_gpu_config1.py)",
          "f32": "north-star topicsMatrix bar NOT met: 4.8e-4 relative on configs[0] (bar 1e-4; one book's ~3300-"
                 "iteration E-step stops at another iterate in fp32); logPerplexity 1e-5 and top-10 terms met "
                 "(tests/test_gpu_config1.py) — a fast secondary mode, not a parity mode",
          "mixed": "north-star bars met: topicsMatrix within 1e-4 relative, logPerplexity within 1e-5, identical "
                   "top-10 terms on configs[0] (tests/test_gpu_config1.py; the fp32 E-step with the documents past "
                   "500 fp32 iterations re-solved in fp64, tests/test_gpu_mixed.py)"}


def summarize(r, a, dtype, world, steps, corpus_kind, kernel):
    """value / roofline / roofline_compute of one run (rank-0 view of the reduced counters).

    roofline window = SURVEY §8(d)'s K6: B_doc counts one gather of each entry's k-wide
    expElogβ' row (the E-step kernel) AND one scatter of its k-wide sstats row, which the separate sstats
    phase performs (radix sort of the (term, slot) keys + the term-sorted k_sstats SpMM), so the bytes are
    divided by the E-step + sstats device time; `phase_split` gives each phase its own bytes and time."""
    estep_ms = r["phases"]["estep"]
    sstats_ms = r["phases"].get("sstats", 0.0)
    window_ms = estep_ms + sstats_ms
    per_step_docs = r["docs_local"] / max(1, steps)
    per_step_nnz = r["entries_local"] / max(1, steps)
    per_step_iters = r["iters_local"] / max(1, steps)
    alg = algorithmic_bytes(per_step_nnz, a.k, per_step_docs, dtype)
    s_b = 8.0 if dtype == "f64" else 4.0
    scatter = per_step_nnz * a.k * s_b  # the sstats rows written (K6's scatter half)
    achieved = alg / (window_ms * 1e-3) / 1e9
    mean_nnz = per_step_nnz / max(1.0, per_step_docs)
    flops = 4.0 * mean_nnz * a.k * per_step_iters
    tflops = flops / (estep_ms * 1e-3) / 1e12
    traffic, traffic_note = pmc_traffic(a, dtype, corpus_kind)
    s = 8 if dtype == "f64" else 4
    return {
        "value": r["docs_all"] / r["elapsed"],
        "ms_per_step": r["elapsed"] * 1e3 / steps,
        "mean_nnz_per_doc": r["entries_all"] / max(1.0, r["docs_all"]),
        "mean_inner_iters": r["iters_all"] / max(1.0, r["docs_all"]),
        "cap_hits": r["cap_hits"],
        "phase_ms": dict({k: round(v, 4) for k, v in r["phases"].items() if k != "steps"},
                         **({"estep_slowest_member": round(r["estep_ms_slowest_member"], 4)}
                            if r.get("estep_ms_slowest_member") is not None else {})),
        "estep_only_docs_per_s": per_step_docs * world / (estep_ms * 1e-3),
        "cold": r["cold"],
        "parity": PARITY[dtype],
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic["window"] if traffic else None,
            "kernel": kernel, "algorithmic_bytes_per_launch": alg,
            "algorithmic_bytes_per_doc": f"nnz*(4+{s}) + 2*nnz*k*{s} + {s}*k",
            "window": "K6 = E-step kernel + sstats phase (radix sort + k_sstats): the gather and the scatter "
                      "B_doc counts; kernel_ms_per_launch is their summed device time per minibatch",
            "kernel_ms_per_launch": window_ms, "traffic_source": traffic_note,
            "phase_split": {
                "estep": {"ms": estep_ms, "algorithmic_bytes": alg - scatter,
                          "traffic": traffic["kernel"] if traffic else None,
                          "GBs": (alg - scatter) / (estep_ms * 1e-3) / 1e9 if estep_ms > 0 else None},
                "sstats": {"ms": sstats_ms, "algorithmic_bytes": scatter,
                           "GBs": scatter / (sstats_ms * 1e-3) / 1e9 if sstats_ms > 0 else None}},
        },
        "roofline_compute": {
            "bound": f"valu_{dtype}", "achieved": tflops, "peak": PEAK_TFS[dtype], "unit": "TFLOP/s",
            "frac": tflops / PEAK_TFS[dtype], "kernel": kernel.split(" ")[0], "flops_per_launch": flops,
            "kernel_ms_per_launch": estep_ms,
        },
    }


KERNEL_TEXT = {
    "k_estep_rows64": "k_estep_rows64_pers (lda_rows64.hip): the fp64 training E-step, one launch per minibatch on a "
                      "resident grid taking document tickets",
    "k_estep_grid": "k_estep_grid_pers (lda_grid.hip): the fp32 training E-step, one launch per minibatch on a resident "
                    "grid taking document tickets",
    "k_estep_tgrid64": "k_estep_tgrid64 (lda_team64.hip): the fp64 many-topic training E-step, a team of CUs per "
                       "document with the topics split (rows64 grid in each member), one launch per minibatch",
    "k_estep_wide_mc": "k_estep_wide_mc (lda_wide.hip): the many-topic training E-step, the rows of a document split "
                       "over a team of CUs, one launch per minibatch",
    "k_estep_wide_tc": "k_estep_wide_tc (lda_wide.hip): the many-topic training E-step, the topics of a document split "
                       "over a team of CUs, one launch per minibatch",
    "k_estep_wide": "k_estep_wide (lda_wide.hip): the many-topic training E-step, one CU per document, one launch per "
                    "minibatch",
    "k_estep": "k_estep (lda.hip): the workgroup E-step for documents past the fast kernels' row capacity",
}


def kernel_name(launched):
    """The training E-step kernel libstc dispatched in the timed steps, from its own launch counters
    (stc_lda_kernel_counts; ADVICE r5: not inferred from k and dtype): the family with the most launches,
    the others (the 7-8-row-set pass, team fallbacks, the workgroup kernel) named beside it."""
    fams = {f: n for f, n in launched.items() if f in KERNEL_TEXT}
    if not fams:
        return "no E-step launch in the timed steps"
    main = max(fams, key=lambda f: fams[f])
    if launched.get("mixed_resolves") and "k_estep_grid" in fams:  # mixed: the fp32 pass is the step's kernel
        main = "k_estep_grid"
    extra = {f: n for f, n in launched.items() if f != main}
    return KERNEL_TEXT[main] + (f"; also launched: {extra}" if extra else "")


def launch_mode(gpus, env, force_group=False):
    """How this process runs N GPUs: "ranks" — one process per GPU under torchrun (WORLD_SIZE set); "group"
    — `python bench.py --gpus N` with no launcher (or --launch group at any N): ONE process drives the N
    devices through stc_group (the reference's own deployment, one JVM on Spark local[*],
    LDATraining.scala:7); "single" — N = 1."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world > 1:
        return "ranks", world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
    if gpus > 1 or force_group:
        return "group", gpus, 0, 0
    return "single", 1, 0, 0


def main():
    a = parse()
    mode, world, rank, local = launch_mode(a.gpus, os.environ, a.launch == "group")
    a.gpus = world
    log = (lambda msg: print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True))  # progress on stderr
    from stc import synth  # no GPU touched yet: the corpus pool may fork

    if a.featurisation_only:
        tokens = synth.token_corpus(a.docs, a.tokens, seed=a.seed + 2, workers=a.workers)
        import stc

        print(json.dumps(featurization(stc, stc.Context(local), a, log, tokens, reps=max(1, a.steps))), flush=True)
        return

    # corpus: strong = rows [r·D/N, (r+1)·D/N) of one corpus; weak = an own D-doc corpus per rank / member.
    # A group is given the whole corpus on the host and shards it itself (contiguous rows, balanced by entries).
    t0 = time.perf_counter()
    if mode == "group":
        workers = max(1, min(a.workers, os.cpu_count() or 1))
        if a.scaling == "strong":
            corpus, total = synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, a.seed, 0, a.docs, workers), a.docs
        else:
            parts = [synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, a.seed + 7919 * r, 0, a.docs, workers)
                     for r in range(world)]
            corpus, total = synth.concat_rows(parts, a.vocab), a.docs * world
            del parts
        lo, hi = 0, corpus.num_rows
    else:
        if a.scaling == "strong":
            lo, hi, seed, total = rank * a.docs // world, (rank + 1) * a.docs // world, a.seed, a.docs
        else:
            lo, hi, seed, total = 0, a.docs, a.seed + 7919 * rank, a.docs * world
        workers = max(1, min(a.workers, (os.cpu_count() or 1)) // max(1, world))
        corpus = synth.make_corpus(a.corpus, a.docs, a.tokens, a.vocab, a.k, seed, lo, hi, workers)
    gen_s = time.perf_counter() - t0
    log(f"{mode}: corpus rows [{lo}, {hi}) generated in {gen_s:.1f} s")
    secondary = world == 1 and not a.no_secondary and mode != "group"  # (the secondary lines run on one context)
    planted = None
    if secondary:
        t0 = time.perf_counter()
        planted = (synth.zipf_lda_corpus(a.docs, a.tokens, a.vocab, a.k, seed=a.seed + 1, workers=workers),
                   synth.planted_topics(a.vocab, a.k, seed=a.seed + 1))
        log(f"planted-topic corpus generated in {time.perf_counter() - t0:.1f} s")
        t0 = time.perf_counter()
        tokens = synth.token_corpus(a.docs, a.tokens, seed=a.seed + 2, workers=workers)
        log(f"token corpus generated in {time.perf_counter() - t0:.1f} s")

    dist = None
    if mode == "ranks":
        import torch.distributed as dist  # control plane only (uid exchange, barrier, max time)

        import datetime

        # a bounded control plane: a rank whose peer died fails its barrier instead of waiting 30 min; the
        # data path's own waits end at STC_COLL_TIMEOUT_MS (api.hip poll_wait) and abort the communicator
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=int(os.environ.get("STC_DIST_TIMEOUT_S", "900"))))
    import stc

    lam_head = None
    if a.state == "planted":
        if a.corpus != "zipf-lda":
            raise SystemExit("--state planted needs --corpus zipf-lda")
        lam_head = synth.planted_topics(a.vocab, a.k, seed=a.seed)
    DT = {"f32": stc.STC_F32, "f64": stc.STC_F64, "mixed": stc.STC_F64}  # (the corpus CSR's value dtype)
    if mode == "group":
        n_dev = stc.Context.device_count()
        if n_dev < world:
            raise SystemExit(f"bench.py --gpus {world}: only {n_dev} device(s) visible; refusing to report "
                             f"{world} GPUs")
        devices = list(range(world))
        log(f"stc_group over devices {devices}")
        model = _Group(stc, a, a.dtype, corpus, devices)
        ctx = None

        def barrier():
            model.sync()
    else:
        ctx = stc.Context(local)
        if mode == "ranks":
            obj = [stc.Context.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.comm_init(obj[0], world, rank)

        def barrier():
            ctx.synchronize()
            if dist is not None:
                dist.barrier()

        dcorp = {a.dtype: stc.DeviceCsr.upload(ctx, corpus, DT[a.dtype])}
        model = _Single(stc, ctx, a, a.dtype, dcorp[a.dtype], total)

    def reduce_run(r):
        el, d, e, it = r["elapsed"], float(r["docs"]), float(r["entries"]), float(r["iters"])
        if dist is not None:
            import torch

            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            s = torch.tensor([d, e, it], dtype=torch.float64)
            dist.all_reduce(s)
            el, (d, e, it) = float(t[0]), (float(x) for x in s)
        r.update(elapsed=el, docs_all=d, entries_all=e, iters_all=it)
        return r

    # the featurisation line first, as the pipeline runs (HashingTF → IDF precede the LDA training,
    # LDAClustering.scala:154-192 → :61), on a device holding only the uploaded corpus
    feat = None
    if secondary:
        log("featurisation")
        feat = featurization(stc, ctx, a, log, tokens)
        del tokens

    r = run_state(model, lam_head, barrier, log, a, a.dtype, a.steps, a.warmup)
    head = summarize(reduce_run(r), a, a.dtype, world, a.steps, a.corpus, kernel_name(r["kernels"]))
    h = model.h

    lines = []
    if secondary:
        other = "f32" if a.dtype == "f64" else "f64"
        dcorp[other] = stc.DeviceCsr.upload(ctx, corpus, DT[other])
        r2 = run_state(_Single(stc, ctx, a, other, dcorp[other], total), None, barrier, log, a, other, a.steps, a.warmup)
        s2 = summarize(reduce_run(r2), a, other, world, a.steps, a.corpus, kernel_name(r2["kernels"]))
        lines.append(dict(label=f"{other} E-step, same corpus and model state", dtype=other, corpus=a.corpus, **s2))
        if a.dtype == "f64":  # the fast mode that meets the north-star bars, on the fp64 corpus upload
            rm = run_state(_Single(stc, ctx, a, "mixed", dcorp["f64"], total), None, barrier, log, a, "mixed",
                           a.steps, a.warmup)
            sm = summarize(reduce_run(rm), a, "mixed", world, a.steps, a.corpus, kernel_name(rm["kernels"]))
            sm["mixed_resolved_docs_per_step"] = rm["kernels"].get("mixed_docs", 0) / max(1, a.steps)
            lines.append(dict(label="mixed E-step (fp32 + fp64 re-solve of the documents past 500 fp32 iterations), "
                                    "same corpus and model state", dtype="mixed", corpus=a.corpus, **sm))
        pc, lam_p = planted
        for dt in (a.dtype, other):
            dp = stc.DeviceCsr.upload(ctx, pc, DT[dt])
            r3 = run_state(_Single(stc, ctx, a, dt, dp, a.docs), lam_p, barrier, log, a, dt, a.steps, a.warmup)
            s3 = summarize(reduce_run(r3), a, dt, world, a.steps, "zipf-lda", kernel_name(r3["kernels"]))
            lines.append(dict(label=f"{dt} E-step, planted-topic corpus at the planted model (SURVEY §8(d) state B)",
                              dtype=dt, corpus="zipf-lda", **s3))
            dp.free()
        dcorp[other].free()
        lines.append(feat)

    if rank != 0:
        if dist is not None:
            dist.barrier()
        return
    copy_gbs = None if a.no_hbm_copy else hbm_copy_gbs(local)
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        log("cpu baseline")
        cpu = cpu_baseline(h, corpus, a)
    roof = dict(head["roofline"], hbm_copy_measured_GBs=copy_gbs,
                note="the E-step iterates a register-resident block (~150 fixed-point iterations per doc at this "
                     "state), so it is VALU-bound and the HBM fraction is small by construction; see "
                     "roofline_compute and the planted-state secondary line")
    parallelism = {"single": "dp1", "ranks": f"dp{world}", "group": f"group{world}"}[mode]
    line = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "docs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": f"synthetic {a.corpus} corpus (seeded, generated in {gen_s:.0f} s), resident in HBM",
        "config": {
            "baseline_config": f"configs[{a.config - 1}]" if world == 1 or a.config != 2 else "configs[2]",
            "workload": f"online LDA minibatch steps: {a.docs} docs x {a.tokens} tokens"
                        f"{' per GPU' if a.scaling == 'weak' else ' sharded over the GPUs'}, V={a.vocab}, k={a.k}, "
                        f"subsamplingRate={a.fraction}",
            "docs": a.docs, "tokens_per_doc": a.tokens, "vocab": a.vocab, "k": a.k,
            "subsampling_rate": a.fraction, "corpus": a.corpus, "parallelism": parallelism,
            "launch": {"single": "one process, one GPU",
                       "ranks": f"{world} processes (torchrun), one GPU each, RCCL communicator via stc_comm_init",
                       "group": f"one process, {world} GPU(s) through stc_group (one host thread per device), "
                                f"collectives: {model.h.transport() if mode == 'group' else ''}"}[mode],
            "mean_nnz_per_doc": head["mean_nnz_per_doc"], "mean_inner_iters": head["mean_inner_iters"],
            "model_state": (f"after {a.state_minibatches} minibatches from lambda0 (Gamma(100,1/100))"
                            if a.state == "burn-in" else
                            f"after {a.state_minibatches} minibatches from the planted topicsMatrix"),
            "cold": head["cold"], "phase_ms": head["phase_ms"],
            "estep_only_docs_per_s": head["estep_only_docs_per_s"], "cap_hits": head["cap_hits"],
        },
        "parity": head["parity"],
        "roofline": roof,
        "roofline_compute": head["roofline_compute"],
        "cpu_baseline": cpu,
        "secondary": lines,
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
