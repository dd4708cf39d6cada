"""Summarise tools/probes/gpu_ab_fetch.sh: bench lines and fetch traffic per variant.
  python tools/probes/ab_report.py VARIANTS CFGS KERNEL_SUBSTR ALG_BYTES"""
import csv
import glob
import json
import sys

variants, cfgs, ksub, alg = sys.argv[1].split(), sys.argv[2].split(), sys.argv[3], float(sys.argv[4])
for v in variants:
    for c in cfgs:
        try:
            for line in open(f"gpurun_out/engab/{v}_{c}.json"):
                if line.startswith("{"):
                    d = json.loads(line)
                    r = d["roofline"]
                    print(v, c, "frac", r["frac"], "us", r["avg_launch_us"], r["kernel"])
        except OSError:
            print(v, c, "missing")
    f = glob.glob(f"gpurun_out/engab/fetch_{v}/**/run_counter_collection.csv", recursive=True)
    if f:
        rows = [r for r in csv.DictReader(open(f[0])) if ksub in r["Kernel_Name"]]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        val = sum(float(r["Counter_Value"]) for r in rows if int(r["Dispatch_Id"]) == last)
        print(v, "fetch x2 / alg", round(val * 2048 / alg, 4))
