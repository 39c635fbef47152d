"""Summarise tools/gpu_prof.sh's rocprofv3 output into profiles/ (committed, read by bench.py).

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
PHASE = re.compile(r"k_estep|k_sstats|k_fixup|rocprim|fillBuffer|k_part_|k_fill_batch|k_batch_nnz")
# the dominant kernel (bench.py's roofline): the training E-step launches (STATS variant), one per
# minibatch — the grid kernel plus the workgroup kernel for the few docs past its row capacity, the
# same launches the bench's HIP-event "estep" phase brackets
# (STATS = true, BOUND = false): k_estep / k_estep_grid / k_estep_wave / k_estep_wide <..., true, false>;
# k_estep_grid64 / k_estep_rows64 <shape, true, false, LONG>; k_estep_wide_mc / _tc <T, Q, NR, true>
ESTEP = re.compile(r"k_estep_grid64<DShape<[^>]*>, true, false, (true|false)>$"  # round-2 profiles
                   r"|k_estep_rows64(_long)?<RShape<[^>]*>, true, false(, (true|false))?>$"
                   r"|k_estep_grid(_long)?<GShape<[^>]*>, true, false(, (true|false))?>$"
                   r"|k_estep_wide_(mc|tc)<\w+, \d+, \d+, true>$"
                   r"|k_estep(_wave|_wide)?<(?!DShape|RShape|GShape).*, true, false>$")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("stc::lda::", "")
    n = re.sub(r"\(.*$", "", n)               # drop the argument list
    n = re.sub(r"^void ", "", n)
    return n[:120]


def load_counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


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
    a = p.parse_args()
    d = a.prof_dir
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    shutil.copy(os.path.join(d, "stats", "stats_kernel_stats.csv"), os.path.join(out_dir, f"{a.tag}_kernel_stats.csv"))

    fetch = load_counters(os.path.join(d, "fetch", "fetch_counter_collection.csv"))
    write = load_counters(os.path.join(d, "write", "write_counter_collection.csv"))
    sq = {}
    sq_path = os.path.join(d, "sq", "sq_counter_collection.csv")
    if os.path.exists(sq_path):
        for kn, cs in load_counters(sq_path).items():
            sq[kn] = {c: sum(v) / len(v) for c, v in cs.items()}

    steps = sum(len(v.get("FETCH_SIZE", [])) for kn, v in fetch.items()
                if kn.startswith("k_lambda_eeb") and kn.endswith(", true>"))
    kernels = {}
    phase_total = 0.0
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
    per_step = phase_total / max(1, steps)
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
    detail = {"workload": wl, "estep_sources_sha": sha, "minibatches_in_run": steps, "kernels": kernels, "sq_per_dispatch": sq,
              "estep_phase_bytes_per_step": per_step, "estep_kernel": sorted(est),
              "estep_kernel_bytes_per_launch": est_bytes}
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
                    "estep_phase_bytes_per_step": per_step, "minibatches_in_run": steps,
                    "note": f"{a.tag}: FETCH_SIZE x2 + WRITE_SIZE per launch of the training E-step kernel "
                            f"(and of the whole E-step phase per minibatch), averaged over {steps} minibatches "
                            f"(incl. burn-in)"})
    with open(tp, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(json.dumps({"minibatches": steps, "estep_kernel_bytes_per_launch": est_bytes,
                      "estep_phase_bytes_per_step": per_step}))
    for kn, v in kernels.items():
        if v["in_estep_phase"]:
            print(f"  {kn[:90]:90s} n={v['dispatches']:4d} fetch×2={v['fetch_bytes_x2_per_dispatch'] / 1e6:9.1f} MB "
                  f"write={v['write_bytes_per_dispatch'] / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
