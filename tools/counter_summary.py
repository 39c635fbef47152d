"""Per-kernel sums of a rocprofv3 --pmc pass (tools/gpu_counters.sh / gpu_icache.sh output), averaged
per dispatch: python tools/counter_summary.py DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+)<(.*?)>\(", name)
    return f"{m.group(1)}<{m.group(2)[:40]}>" if m else name[:60]


for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        agg, disp = collections.defaultdict(float), collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        print(f)
        for (k, c), v in sorted(agg.items()):
            print(f"  {k:55s} {c:36s} {v / max(1, len(disp[k])):16.4g} per dispatch ({len(disp[k])})")
