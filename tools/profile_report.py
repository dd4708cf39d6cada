"""Turn a tools/gpu_profile.sh run (gpurun_out/prof) into the committed profiles/.

  python tools/profile_report.py --round r03 --prof gpurun_out/prof3

Writes
  profiles/<round>_bench_kernel_stats.csv   rocprofv3 --stats of `python3 bench.py --gpus 1
                                            --steps 20 --warmup 5` (the driver's command)
  profiles/<round>_bench.json               the bench line of that same traced run
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


ENG = ("engine_tri_kernel", "engine_tri_x_kernel", "engine_kernel")
KERNELS = {"c2": ENG, "c3": ENG, "c4": ENG, "c4_noor": ENG, "c4_pe": ENG,
           "c5": ("cgr_stream_kernel", "span_first_kernel"),
           "c5_valid": ("cgr_stream_kernel", "span_first_kernel"),
           "c2_lr": ENG, "c2_250": ENG, "c2_noor": ENG,
           "c2_kmers": ("kmer_tile_kernel", "kmer_maxlen_kernel", "kmer_reduce_kernel")}


def counters(sub, kerns):
    """Per-launch sums: the last dispatch of every kernel the library call runs."""
    if isinstance(kerns, str):
        kerns = (kerns,)
    f = glob.glob(os.path.join(PROF, sub, "**", "run_counter_collection.csv"), recursive=True)
    if not f:
        return {}, None
    rows = [r for r in csv.DictReader(open(f[0])) if any(k in r["Kernel_Name"] for k in kerns)]
    if not rows:
        return {}, None
    last = {}
    for r in rows:
        last[r["Kernel_Name"]] = max(last.get(r["Kernel_Name"], -1), int(r["Dispatch_Id"]))
    agg = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == last[r["Kernel_Name"]]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return dict(agg), " + ".join(sorted(last))


def clock_check(stats_csv, line, kerns):
    """the traced kernel time must fit the SAME run's bench
    clock.  The dominant kernel (largest total in the trace's --stats) averaged
    over the TIMED launches (the last steps x launches-per-step of the kernel
    trace beside the stats file; the untimed warmup's first launches run at a
    lower clock) x launches per step must be <= the line's ms_per_step, else
    the profile is marked box_mismatch (a trace from a slower box than the
    line, or a line that is not this run's)."""
    if not (stats_csv and line):
        return None
    rows = [r for r in csv.DictReader(open(stats_csv)) if any(k in r["Name"] for k in kerns)]
    if not rows:
        return None
    dom = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    c = line["config"]
    per_step = -(-int(c.get("reads_per_gpu", 0)) // max(1, int(c.get("batch_reads", 1))))
    avg, launches = float(dom["AverageNs"]), "all launches (--stats)"
    tr = glob.glob(os.path.join(os.path.dirname(stats_csv), "*kernel_trace.csv"))
    if tr:
        d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                   for r in csv.DictReader(open(tr[0])) if r["Kernel_Name"] == dom["Name"])
        k = int(line["steps"]) * per_step
        if len(d) >= k:
            avg, launches = sum(x for _, x in d[-k:]) / k, f"the last {k} launches (the timed steps)"
    k_ms = avg * per_step / 1e6
    ok = k_ms <= float(line["ms_per_step"]) * 1.0005
    return {"kernel": dom["Name"][:120], "kernel_avg_us": round(avg / 1e3, 2), "averaged_over": launches,
            "launches_per_step": per_step, "kernel_ms_per_step": round(k_ms, 4),
            "bench_ms_per_step": line["ms_per_step"], "device": c.get("device"),
            "status": "consistent" if ok else "box_mismatch"}


def bench_line(path):
    if not os.path.exists(path):
        return None
    lines = open(path).read().strip().splitlines()
    return json.loads(lines[-1]) if lines else None


def config_record(rnd, cfg):
    b = bench_line(os.path.join(PROF, f"bench_{cfg}.json"))
    fetch, kname = counters(f"fetch_{cfg}", KERNELS[cfg])
    write, _ = counters(f"write_{cfg}", KERNELS[cfg])
    if not (b and fetch and write):
        return None
    rec = {"round": rnd, "config": cfg, "kernel_symbols": kname,
           "batch_reads": b["config"]["batch_reads"], "kernel": b["roofline"]["kernel"],
           "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"],
           "source": "tools/gpu_profile.sh; rocprofv3 --kernel-trace --pmc, one counter per pass, "
                     "last dispatch of each kernel of one library call (tools/prof_engine.py)",
           "FETCH_SIZE_kB": fetch.get("FETCH_SIZE"), "fetch_bytes_x2": int(fetch["FETCH_SIZE"] * 1024 * 2),
           "WRITE_SIZE_kB": write.get("WRITE_SIZE"), "write_bytes": int(write["WRITE_SIZE"] * 1024)}
    rec["hbm_bytes_per_launch"] = rec["fetch_bytes_x2"] + rec["write_bytes"]
    rec["traffic_over_alg"] = round(rec["hbm_bytes_per_launch"] / rec["alg_bytes_per_launch"], 4)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--kernel", default="engine_tri_kernel")
    ap.add_argument("--prof", default=None, help="profile output dir (default gpurun_out/prof)")
    a = ap.parse_args()
    global PROF
    if a.prof:
        PROF = os.path.join(ROOT, a.prof) if not os.path.isabs(a.prof) else a.prof
    os.makedirs(OUT, exist_ok=True)
    stats = glob.glob(os.path.join(PROF, "trace", "**", "run_kernel_stats.csv"), recursive=True)
    main_check = clock_check(stats[0] if stats else None, bench_line(os.path.join(PROF, "bench.json")), ENG)
    if main_check:
        print("clock check (driver command):", json.dumps(main_check))
        if main_check["status"] != "consistent":
            raise SystemExit("profile_report: the kernel trace does not fit its own bench clock (box_mismatch)")
    if stats:
        shutil.copy(stats[0], os.path.join(OUT, f"{a.round}_bench_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if a.kernel in r["Name"]:
                print("kernel-trace avg ns:", r["AverageNs"], "calls", r["Calls"])
    b = bench_line(os.path.join(PROF, "bench.json"))
    if b and main_check:
        b["clock_check"] = main_check
    if b:
        json.dump(b, open(os.path.join(OUT, f"{a.round}_bench.json"), "w"), indent=1)
        print("bench value", b["value"], "avg_launch_us", b["roofline"]["avg_launch_us"])
    for cfg in KERNELS:
        rec = config_record(a.round, cfg)
        if rec is None:
            continue
        if cfg == "c2":
            sq1, _ = counters("sq1", a.kernel)
            sq2, _ = counters("sq2", a.kernel)
            rec["sq"] = {**sq1, **sq2}
        if cfg in ("c5", "c5_valid"):   # LDS bound of the CGR stream pass
            mode = "cgr" if cfg == "c5" else "cgrv"
            l1, _ = counters(f"lds1_{mode}", "cgr_stream_kernel")
            l2, _ = counters(f"lds2_{mode}", "cgr_stream_kernel")
            if l1 or l2:
                rec["sq"] = {**l1, **l2}
                if l2.get("SQ_LDS_IDX_ACTIVE"):
                    rec["lds_conflict_ratio"] = round(l2["SQ_LDS_BANK_CONFLICT"] / l2["SQ_LDS_IDX_ACTIVE"], 4)
        if cfg == "c2_kmers":   # LDS banks and the texture addresser
            l2, _ = counters("lds2_kmers", "kmer_tile_kernel")
            ta, _ = counters("ta_kmers", "kmer_tile_kernel")
            if l2 or ta:
                rec["sq"] = {**l2, **ta}
                if l2.get("SQ_LDS_IDX_ACTIVE"):
                    rec["lds_conflict_ratio"] = round(l2["SQ_LDS_BANK_CONFLICT"] / l2["SQ_LDS_IDX_ACTIVE"], 4)
                if ta.get("GRBM_GUI_ACTIVE"):   # GRBM sums 8 XCDs, TA_TA_BUSY_sum 256 CUs
                    rec["ta_busy_frac"] = round(ta["TA_TA_BUSY_sum"] / 256 / (ta["GRBM_GUI_ACTIVE"] / 8), 4)
        # the bench lines of this session carry THIS session's PMC bytes (bench.py
        # copies whatever profiles/pmc_engine_<cfg>.json held when it ran, which
        # is the previous session's: VERDICT r4 item 7)
        src = (f"profiles/{a.round}_pmc_engine_{cfg}.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
               "separate passes, same session)")
        cb = bench_line(os.path.join(PROF, f"bench_{cfg}.json"))
        bt = glob.glob(os.path.join(PROF, f"btrace_{cfg}", "**", "run_kernel_stats.csv"), recursive=True)
        chk = clock_check(bt[0] if bt else None, cb, KERNELS[cfg])
        if cb and chk:
            cb["clock_check"] = chk
            if chk["status"] != "consistent":
                print(f"{cfg}: BOX MISMATCH", json.dumps(chk))
        if cb:
            cb["roofline"]["traffic"] = rec["hbm_bytes_per_launch"]
            cb["roofline"]["traffic_source"] = src
            json.dump(cb, open(os.path.join(OUT, f"{a.round}_bench_{cfg}.json"), "w"), indent=1)
        if cfg == "c2" and b:
            b["roofline"]["traffic"] = rec["hbm_bytes_per_launch"]
            b["roofline"]["traffic_source"] = src
            json.dump(b, open(os.path.join(OUT, f"{a.round}_bench.json"), "w"), indent=1)
        if bt:
            shutil.copy(bt[0], os.path.join(OUT, f"{a.round}_bench_{cfg}_kernel_stats.csv"))
        for name in (f"{a.round}_pmc_engine_{cfg}.json", f"pmc_engine_{cfg}.json"):
            json.dump(rec, open(os.path.join(OUT, name), "w"), indent=1)
        print(cfg, json.dumps({k: v for k, v in rec.items() if k != "sq"}))


if __name__ == "__main__":
    main()
