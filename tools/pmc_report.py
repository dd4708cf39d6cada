"""Summarise rocprofv3 --pmc CSVs for one kernel (per dispatch, last dispatch)."""
import collections
import csv
import glob
import sys

kern = sys.argv[2] if len(sys.argv) > 2 else "engine_kernel"
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    last = None
    for r in rows:
        if kern not in r["Kernel_Name"]:
            continue
        last = r["Dispatch_Id"]
    for r in rows:
        if kern in r["Kernel_Name"] and r["Dispatch_Id"] == last:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    for c, v in sorted(agg.items()):
        print(f"{f.split('/')[-2]:4s} {c:24s} {v:16.0f}")
