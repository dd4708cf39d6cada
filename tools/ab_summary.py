"""Summarise a tools/gpu_run.sh session: per variant and config the bench
lines (launch time, roofline fraction; mean / min over the alternating rounds)
and the PMC traffic (FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 per launch,
MI355X_MICROARCH.md HBM section; last dispatch of each kernel of the call).

  python tools/ab_summary.py gpurun_out/TAG [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

ENG = ("engine_tri_kernel", "engine_tri_x_kernel", "engine_kernel")
KERNELS = collections.defaultdict(lambda: ENG, {
    "c5": ("cgr_stream_kernel", "span_first_kernel"),
    "c5_valid": ("cgr_stream_kernel", "span_first_kernel"),
    "c2_kmers": ("kmer_tile_kernel", "kmer_maxlen_kernel", "kmer_reduce_kernel")})


def pmc(d, kerns):
    f = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
    if not f:
        return None
    rows = [r for r in csv.DictReader(open(f[0])) if any(k in r["Kernel_Name"] for k in kerns)]
    last = {}
    for r in rows:
        last[r["Kernel_Name"]] = max(last.get(r["Kernel_Name"], -1), int(r["Dispatch_Id"]))
    agg = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == last[r["Kernel_Name"]]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return dict(agg)


def main():
    top = sys.argv[1]
    out = {}
    for f in sorted(glob.glob(os.path.join(top, "bench_*.jsonl"))):
        name, cfg = os.path.basename(f)[6:-6].split("_", 1)
        lines = [json.loads(x) for x in open(f) if x.startswith("{")]
        us = [x["roofline"]["avg_launch_us"] for x in lines]
        fr = [x["roofline"]["frac"] for x in lines]
        rec = out.setdefault(f"{name} {cfg}", {})
        rec.update(runs=len(us), us=us, us_mean=round(sum(us) / len(us), 1), us_min=min(us),
                   frac_mean=round(sum(fr) / len(fr), 4), frac_max=max(fr),
                   kernel=lines[0]["roofline"]["kernel"],
                   alg=lines[0]["roofline"]["alg_bytes_per_launch"])
    for d in sorted(glob.glob(os.path.join(top, "pmc_*_FETCH_SIZE"))):
        name, cfg = os.path.basename(d)[4:-len("_FETCH_SIZE")].split("_", 1)
        fe = pmc(d, KERNELS[cfg])
        wr = pmc(d.replace("FETCH_SIZE", "WRITE_SIZE"), KERNELS[cfg])
        if not fe or not wr:
            continue
        rec = out.setdefault(f"{name} {cfg}", {})
        rec["fetch_bytes_x2"] = int(fe["FETCH_SIZE"] * 2048)
        rec["write_bytes"] = int(wr["WRITE_SIZE"] * 1024)
        rec["hbm_bytes"] = rec["fetch_bytes_x2"] + rec["write_bytes"]
        if "alg" in rec:
            rec["traffic_over_alg"] = round(rec["hbm_bytes"] / rec["alg"], 4)
    for d in sorted(glob.glob(os.path.join(top, "sq1_*"))):
        if not os.path.isdir(d):
            continue
        key = os.path.basename(d)[4:]
        cfg = key.split("_", 1)[1] if key.split("_", 1)[0] not in KERNELS and "_" in key and \
            key.split("_", 1)[1] in ("c2", "c3", "c4", "c4_pe", "c4_noor", "c5", "c5_valid", "c2_kmers") else key
        name = key[:-len(cfg) - 1] if cfg != key else "base"
        a = pmc(d, KERNELS[cfg]) or {}
        b = pmc(d.replace("sq1_", "sq2_"), KERNELS[cfg]) or {}
        rec = out.setdefault(f"{name} {cfg}", {})
        rec["sq"] = {**a, **b}
    for k, v in out.items():
        print(k, {x: y for x, y in v.items() if x not in ("us",)})
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
