"""Summarise tools/gpu.sh feat's FETCH_SIZE / WRITE_SIZE passes of the featurisation line into
profiles/<tag>_featurisation_pmc.json (read by bench.py's featurisation line as `traffic`).

  python tools/feat_pmc_summary.py gpurun_out/featpmc --tag r04

Per kernel: HBM bytes per dispatch = FETCH_SIZE x 2 (the gfx950 correction, MI355X_MICROARCH.md) +
WRITE_SIZE, both rocprofv3 derived counters in KiB, from separate passes.  Stages: HashingTF = the
single pass (or the sorted-key passes) + its memsets; IDF fit = the df count, its reduction and the
hot-idf table; transform = the TF·IDF kernel.  The entry carries the hash of the featurisation sources
(bench.py FEAT_SOURCES): bench reports null traffic when the tree's sources differ.
"""
import argparse
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STAGES = {
    "hashing_tf": re.compile(r"k_doc_hash_emit|k_doc_hash_sort|k_doc_sort|k_doc_runs|k_hash<|k_large_segments"),
    "idf_fit": re.compile(r"k_df_|k_idf|k_keys|k_runs"),
    "idf_transform": re.compile(r"k_transform"),
}


def short(name):
    n = re.sub(r"\(.*$", "", name)
    return re.sub(r"^void ", "", n)


def load(path, counter):
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("prof_dir")
    p.add_argument("--tag", default="r04")
    a = p.parse_args()
    fetch = load(os.path.join(a.prof_dir, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(a.prof_dir, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for kn in sorted(set(fetch) | set(write)):
        fr, wr = fetch.get(kn, []), write.get(kn, [])
        kernels[kn] = {"dispatches": max(len(fr), len(wr)),
                       "fetch_x2_per_dispatch": 2.0 * sum(fr) / max(1, len(fr)),
                       "write_per_dispatch": sum(wr) / max(1, len(wr))}
    stages = {}
    for st, rx in STAGES.items():
        ks = {kn: v for kn, v in kernels.items() if rx.search(kn)}
        if not ks:
            raise SystemExit(f"no kernel of stage {st} among {sorted(kernels)[:10]}: refusing to write")
        stages[st] = {"kernels": sorted(ks),
                      "bytes_per_call": sum(v["fetch_x2_per_dispatch"] + v["write_per_dispatch"] for v in ks.values())}
    from bench import feat_sources_sha

    out = {"tag": a.tag, "feat_sources_sha": feat_sources_sha(), "stages": stages, "kernels": kernels,
           "note": "FETCH_SIZE x2 + WRITE_SIZE per dispatch (separate rocprofv3 --pmc passes), summed per stage"}
    path = os.path.join(ROOT, "profiles", f"{a.tag}_featurisation_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: round(v["bytes_per_call"] / 1e9, 3) for k, v in stages.items()}))


if __name__ == "__main__":
    main()
