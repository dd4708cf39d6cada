"""Turn a tools/gpu_profile.sh run (gpurun_out/prof) into the committed profiles/.

  python tools/profile_report.py --round r01

Writes
  profiles/<round>_bench_kernel_stats.csv   rocprofv3 --stats of `bench.py --steps 5`
  profiles/<round>_bench.json               the bench line of that round's profile run
  profiles/<round>_pmc_engine_c2.json        per-launch PMC summary (FETCH/WRITE/SQ)
  profiles/pmc_engine_c2.json                the latter, read by bench.py for `traffic`
HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KB) x 1024 x 2
on gfx950 (it reports half the bytes of a streaming read), WRITE_SIZE (KB) x
1024 as is; separate passes; last dispatch of the engine kernel.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")
OUT = os.path.join(ROOT, "profiles")


def counters(sub, kern):
    f = glob.glob(os.path.join(PROF, sub, "**", "run_counter_collection.csv"), recursive=True)
    if not f:
        return {}, None
    rows = [r for r in csv.DictReader(open(f[0])) if kern in r["Kernel_Name"]]
    if not rows:
        return {}, None
    last = max(int(r["Dispatch_Id"]) for r in rows)
    agg = collections.defaultdict(float)
    name = None
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            name = r["Kernel_Name"]
    return dict(agg), name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--kernel", default="engine_tri_kernel")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    stats = glob.glob(os.path.join(PROF, "trace", "**", "run_kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(OUT, f"{a.round}_bench_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if a.kernel in r["Name"]:
                print("kernel-trace avg ns:", r["AverageNs"], "calls", r["Calls"])
    bench = os.path.join(PROF, "bench.json")
    if os.path.exists(bench):
        line = open(bench).read().strip().splitlines()[-1]
        b = json.loads(line)
        json.dump(b, open(os.path.join(OUT, f"{a.round}_bench.json"), "w"), indent=1)
        print("bench value", b["value"], "avg_launch_us", b["roofline"]["avg_launch_us"])
    else:
        b = None
    fetch, kname = counters("fetch", a.kernel)
    write, _ = counters("write", a.kernel)
    sq1, _ = counters("sq1", a.kernel)
    sq2, _ = counters("sq2", a.kernel)
    rec = {"round": a.round, "kernel_symbol": kname, "batch_reads": 10_000_000,
           "source": "tools/gpu_profile.sh; rocprofv3 --kernel-trace --pmc, one counter group "
                     "per pass, last dispatch of tools/prof_engine.py --mode c2"}
    if b:
        rec["kernel"] = b["roofline"]["kernel"]
        rec["alg_bytes_per_launch"] = b["roofline"]["alg_bytes_per_launch"]
    if fetch:
        rec["FETCH_SIZE_kB"] = fetch.get("FETCH_SIZE")
        rec["fetch_bytes_x2"] = int(fetch["FETCH_SIZE"] * 1024 * 2)
    if write:
        rec["WRITE_SIZE_kB"] = write.get("WRITE_SIZE")
        rec["write_bytes"] = int(write["WRITE_SIZE"] * 1024)
    if fetch and write:
        rec["hbm_bytes_per_launch"] = rec["fetch_bytes_x2"] + rec["write_bytes"]
        if b:
            rec["traffic_over_alg"] = round(rec["hbm_bytes_per_launch"] / rec["alg_bytes_per_launch"], 4)
    rec["sq"] = {**sq1, **sq2}
    for name in (f"{a.round}_pmc_engine_c2.json", "pmc_engine_c2.json"):
        json.dump(rec, open(os.path.join(OUT, name), "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "sq"}, indent=1))


if __name__ == "__main__":
    main()
