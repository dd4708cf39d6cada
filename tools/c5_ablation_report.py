"""Summarise tools/gpu_c5_ablation_r04.sh (gpurun_out/c5abl) into one JSON:
per variant the bench line's HIP-event time per launch (two runs) and the
per-launch counters of the last cgr_stream_kernel dispatch.

  python tools/c5_ablation_report.py gpurun_out/c5abl > profiles/r04_c5_ablation.json
"""
import collections
import csv
import glob
import json
import os
import sys

VARIANTS = {
    "base": "the product kernel (cgr_stream_kernel<7, false>)",
    "1": "no table add: a VALU xor into a register instead of the ds_add_u64",
    "2": "the quality window chain replaced by a constant",
    "3": "no emission mask: every byte adds to its word's cell",
    "4": "a 32-bit ds_add_u32 of the count only",
    "5": "(exact) bytes that end no word skip the add by EXEC masking, no spare-cell adds",
}


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if "cgr_stream_kernel" in r["Kernel_Name"]]
        if not rows:
            continue
        last = max(int(r["Dispatch_Id"]) for r in rows)
        agg = collections.defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
        out.update(agg)
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5abl"
    res = {"what": "C5 (k = 7, 5 M x 250 bp per call) timing-only ablations of the stream kernel's per-byte "
                   "loop, one box, one call (tools/gpu_c5_ablation_r04.sh); counters are per launch "
                   "(last dispatch), summed over the chip", "variants": {}}
    for v, desc in VARIANTS.items():
        us = []
        for f in sorted(glob.glob(os.path.join(root, f"bench_{v}_*.json"))):
            try:
                us.append(json.loads(open(f).read().strip().splitlines()[-1])["roofline"]["avg_launch_us"])
            except (ValueError, IndexError, KeyError):
                pass
        c = counters(os.path.join(root, f"pmc_{v}"))
        c.update(counters(os.path.join(root, f"pmc2_{v}")))
        rec = {"desc": desc, "avg_launch_us": us, "counters": {k: int(x) for k, x in sorted(c.items())}}
        if c.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_conflict_ratio"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 3)
        res["variants"][v] = rec
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
