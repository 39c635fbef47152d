"""Summarise tools/gpu.sh prof's rocprofv3 output into profiles/ (committed, read by bench.py).

  python tools/pmc_summary.py gpurun_out/prof --docs 1000000 --tokens 200 --vocab 262144 --k 100 \
      --fraction 0.05 --corpus zipf --tag r01

Writes:
  profiles/<tag>_kernel_stats.csv   the --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.json           per-kernel FETCH/WRITE bytes + SQ counters per dispatch
  profiles/pmc_traffic.json         per workload: E-step HBM bytes per launch (bench.py's `traffic`)

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB from the L2's fabric-side request
counters, measured in SEPARATE --pmc passes (they do not fit one pass on gfx950).  On gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads, so it is doubled
(MI355X_MICROARCH.md, HBM section).  Infinity-Cache hits are counted as fabric traffic.
One minibatch = one UPDATE=true dispatch of the fused M-step pass (k_lambda_eeb / k_lambda_eeb_wide).
"""
import argparse
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# kernels of the E-step phase (the bench roofline's "kernel"): E-step, term sort, sstats SpMM,
# the stat memset, and the partition scans (rocprim; tiny)
PHASE = re.compile(r"k_estep|k_sstats|k_fixup|rocprim|fillBuffer|k_part_|k_fill_batch|k_batch_nnz|k_mixed_|k_entry_pairs")
# bench.py's roofline window (SURVEY §8(d) K6 = gather + scatter): the training E-step launches and the
# sstats phase after them — the stat clear, the (term, slot) radix sort, k_sstats / k_fixup, logphat and the
# iteration statistics (HIP events 1 → 3 in api.hip estep_and_stats)
WINDOW = re.compile(r"k_estep|k_rows64_long_list|k_sstats|k_fixup|k_logphat|k_iter_stats|fillBuffer"
                    r"|radix_sort_onesweep|k_mixed_|k_entry_pairs")  # (k_mixed_: the mixed mode's fp64 re-solve list and
# fixup; k_entry_pairs: the fp64 rows path's sstats pairs, built beside the E-step since round 6)
# the dominant kernel (bench.py's roofline): the training E-step launches (STATS variant), one per
# minibatch — the grid kernel plus the workgroup kernel for the few docs past its row capacity, the
# same launches the bench's HIP-event "estep" phase brackets
# (STATS = true, BOUND = false): k_estep / k_estep_grid / k_estep_wave / k_estep_wide <..., true, false>;
# k_estep_grid64 / k_estep_rows64[_long|_pers] / k_estep_grid[_long|_pers] <shape, true, false, LONG>; k_estep_wide_mc / _tc <T, Q, NR, true>
ESTEP = re.compile(r"k_estep_grid64<DShape<[^>]*>, true, false, (true|false)>$"  # round-2 profiles
                   r"|k_estep_rows64(_long|_pers)?<RShape<[^>]*>, true, false(, (true|false))?>$"
                   r"|k_estep_grid(_long|_pers)?<GShape<[^>]*>, true, false(, (true|false))?>$"
                   r"|k_estep_wide_(mc|tc)<\w+, \d+, \d+, true>$"
                   r"|k_estep_tgrid64<\d+, true>$"
                   r"|k_estep(_wave|_wide)?<(?!DShape|RShape|GShape).*, true, false>$")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("stc::lda::", "")
    n = re.sub(r"\(.*$", "", n)               # drop the argument list
    n = re.sub(r"^void ", "", n)
    return n[:120]


def _last(rows, keep_frac):
    """the last ceil(len·keep_frac) rows by dispatch id (the steady-state minibatches' dispatches)"""
    if keep_frac >= 1.0:
        return rows
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    n = max(1, int(round(len(rows) * keep_frac)))
    return rows[-n:]


def load_counters(path, keep_frac=1.0):
    by = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            by[(short(r["Kernel_Name"]), r["Counter_Name"])].append(r)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (kn, cn), rows in by.items():
        agg[kn][cn] = [float(r["Counter_Value"]) for r in _last(rows, keep_frac)]
    return agg


def steady_stats(trace_csv, out_csv, keep_frac):
    """--kernel-trace dispatches → a stats table in rocprofv3's --stats format over the last keep_frac of
    every kernel's dispatches (the timed minibatches: the bench runs burn-in first, whose cold launches
    iterate longer), so its averages reproduce the bench's per-launch times."""
    by = collections.defaultdict(list)
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            by[r["Kernel_Name"]].append(r)
    rows = []
    for kn, rs in by.items():
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in _last(rs, keep_frac)]
        tot = sum(d)
        mean = tot / len(d)
        sd = (sum((x - mean) ** 2 for x in d) / len(d)) ** 0.5
        rows.append((kn, len(d), tot, mean, min(d), max(d), sd))
    grand = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for kn, n, tot, mean, mn, mx, sd in rows:
            w.writerow([kn, n, tot, mean, 100.0 * tot / grand, mn, mx, sd])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof_dir")
    p.add_argument("--docs", type=int, default=1_000_000)
    p.add_argument("--tokens", type=int, default=200)
    p.add_argument("--vocab", type=int, default=1 << 18)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--fraction", type=float, default=0.05)
    p.add_argument("--corpus", default="zipf")
    p.add_argument("--dtype", default="f64")
    p.add_argument("--tag", default="r01")
    p.add_argument("--steady", type=int, default=0,
                   help="summarise only the last N minibatches (the bench's timed steps; 0 = every dispatch)")
    p.add_argument("--minibatches", type=int, default=0,
                   help="minibatches the profiled run made (needed with --steady: 3 cold + burn-in + warmup + steps)")
    a = p.parse_args()
    d = a.prof_dir
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    keep = 1.0
    if a.steady:
        if a.minibatches <= 0:
            raise SystemExit("--steady needs --minibatches")
        keep = a.steady / a.minibatches
        steady_stats(os.path.join(d, "stats", "stats_kernel_trace.csv"), os.path.join(out_dir, f"{a.tag}_kernel_stats.csv"),
                     keep)
    else:
        shutil.copy(os.path.join(d, "stats", "stats_kernel_stats.csv"), os.path.join(out_dir, f"{a.tag}_kernel_stats.csv"))

    fetch = load_counters(os.path.join(d, "fetch", "fetch_counter_collection.csv"), keep)
    write = load_counters(os.path.join(d, "write", "write_counter_collection.csv"), keep)
    sq = {}
    sq_path = os.path.join(d, "sq", "sq_counter_collection.csv")
    if os.path.exists(sq_path):
        for kn, cs in load_counters(sq_path, keep).items():
            sq[kn] = {c: sum(v) / len(v) for c, v in cs.items()}

    steps = sum(len(v.get("FETCH_SIZE", [])) for kn, v in fetch.items()
                if kn.startswith("k_lambda_eeb") and kn.endswith(", true>"))
    kernels = {}
    phase_total = 0.0
    window_total = 0.0
    for kn in sorted(set(fetch) | set(write)):
        fr = fetch.get(kn, {}).get("FETCH_SIZE", [])
        wr = write.get(kn, {}).get("WRITE_SIZE", [])
        f_raw = sum(fr) * 1024.0
        w_b = sum(wr) * 1024.0
        kernels[kn] = {
            "dispatches": max(len(fr), len(wr)),
            "fetch_bytes_raw_per_dispatch": f_raw / max(1, len(fr)),
            "fetch_bytes_x2_per_dispatch": 2.0 * f_raw / max(1, len(fr)),
            "write_bytes_per_dispatch": w_b / max(1, len(wr)),
            "in_estep_phase": bool(PHASE.search(kn)),
        }
        if PHASE.search(kn):
            phase_total += 2.0 * f_raw + w_b
        if WINDOW.search(kn):
            window_total += 2.0 * f_raw + w_b
    per_step = phase_total / max(1, steps)
    window_per_step = window_total / max(1, steps)
    est = {kn: v for kn, v in kernels.items() if ESTEP.search(kn)}
    est_launches = max((v["dispatches"] for v in est.values()), default=0)
    est_bytes = sum((v["fetch_bytes_x2_per_dispatch"] + v["write_bytes_per_dispatch"]) * v["dispatches"]
                    for v in est.values()) / max(1, est_launches)
    if not est or est_bytes <= 0:
        raise SystemExit(f"no training E-step kernel matched among {sorted(kernels)[:12]}: refusing to write "
                         f"an empty traffic entry (fix ESTEP)")
    from bench import estep_sources_sha

    sha = estep_sources_sha()
    wl = {"docs": a.docs, "tokens": a.tokens, "vocab": a.vocab, "k": a.k, "fraction": a.fraction,
          "corpus": a.corpus, "dtype": a.dtype}
    span = (f"the last {steps} minibatches (the timed steady state) of {a.minibatches}" if a.steady
            else f"{steps} minibatches (incl. burn-in)")
    detail = {"workload": wl, "estep_sources_sha": sha, "minibatches_in_run": steps, "window": span,
              "kernels": kernels, "sq_per_dispatch": sq,
              "estep_phase_bytes_per_step": per_step, "k6_window_bytes_per_step": window_per_step,
              "estep_kernel": sorted(est), "estep_kernel_bytes_per_launch": est_bytes}
    with open(os.path.join(out_dir, f"{a.tag}_pmc.json"), "w") as f:
        json.dump(detail, f, indent=1)
    # pmc_traffic.json holds one entry per workload (bench.py picks the one matching its run)
    tp = os.path.join(out_dir, "pmc_traffic.json")
    try:
        with open(tp) as f:
            entries = json.load(f)
        entries = entries.get("entries", [entries]) if isinstance(entries, dict) else entries
    except (OSError, ValueError):
        entries = []
    entries = [e for e in entries if e.get("workload") != wl]
    entries.append({"workload": wl, "tag": a.tag, "estep_sources_sha": sha,
                    "estep_kernel": sorted(est), "estep_kernel_bytes_per_launch": est_bytes,
                    "estep_phase_bytes_per_step": per_step, "k6_window_bytes_per_step": window_per_step,
                    "minibatches_in_run": steps,
                    "note": f"{a.tag}: FETCH_SIZE x2 + WRITE_SIZE per minibatch of the K6 window (E-step kernel + "
                            f"sstats phase) and per launch of the E-step kernel, averaged over {span}"})
    with open(tp, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(json.dumps({"minibatches": steps, "estep_kernel_bytes_per_launch": est_bytes,
                      "estep_phase_bytes_per_step": per_step, "k6_window_bytes_per_step": window_per_step}))
    for kn, v in kernels.items():
        if v["in_estep_phase"]:
            print(f"  {kn[:90]:90s} n={v['dispatches']:4d} fetch×2={v['fetch_bytes_x2_per_dispatch'] / 1e6:9.1f} MB "
                  f"write={v['write_bytes_per_dispatch'] / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
