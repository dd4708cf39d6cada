#!/usr/bin/env python3
"""bench.py — hpg-fastq hot path on MI355X.

Default workload (BASELINE.json configs[1]): `hpg-fastq stats
--read-quality-range 20, --read-length-range 50,` over 100 M synthetic 150 bp
single-end reads PER GPU, resident in HBM (10 batches of 10 M reads, the
reference's fastq_batch_t layout).  One step = reset counters + the fused
edit->filter->stats kernel over every batch (+ one RCCL all-reduce of the
packed counters when N > 1).  Reads shard by index across ranks with no
data-path collective: weak scaling.

Other configs (--config; parity cases of BASELINE.json, reported in DESIGN.md,
not the driver's line):
  c3  paired-end 2x150, pair-consistent filter, 100 M pairs per GPU
  c4  edit (5'/3' Q20 trim) + stats, 500 M x 150 over 8 GPUs = 62.5 M per GPU
  c5  chaos game k=7, 200 M x 250 over 8 GPUs = 25 M per GPU

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`--gpus N` with N > 1 and no WORLD_SIZE in the environment starts the N rank
processes itself (fresh interpreters, one per GPU, before this process touches
the GPU) and relays rank 0's line; under torch.distributed.run each rank checks
that WORLD_SIZE equals --gpus.  Rank control (rendezvous, barriers, the
max-over-ranks time) runs on gloo; the data path's one exchange is libhpgq's
RCCL all-reduce, whose rank count is reported as config.rccl_ranks.
`--launch-dry-run` exercises the launcher and the read sharding on CPU (no GPU).

Prints ONE JSON line (rank 0) with `roofline` (the hot kernel, HIP events on
the engine's own stream) and `cpu_baseline` (oracle/liboracle.so, C+OpenMP,
timed on this host's cores on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import ctypes as C
import datetime
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hpg-fastq_amd"))

H = None   # hpgfastq, imported by the rank processes (the launcher never loads libhpgq)


def _load_hpgfastq():
    global H
    if H is None:
        import hpgfastq
        H = hpgfastq
    return H

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)

CONFIGS = {
    "c2": dict(metric="Mreads/s (150 bp) stats+filter at 1/2/4/8 MI355X; achieved HBM GB/s vs peak",
               unit="Mreads/s", reads=100_000_000, batch=10_000_000, L=150, seed=2,
               workload="C2: stats+filter --read-quality-range 20, --read-length-range 50,"),
    "c3": dict(metric="Mpairs/s (2x150 bp) paired-end stats+filter, pair-consistent",
               unit="Mpairs/s", reads=100_000_000, batch=10_000_000, L=150, seed=3,
               workload="C3: PE 2x150 stats+filter --read-quality-range 20, "
                        "--read-length-range 50, (pair passes iff both mates pass)"),
    "c4": dict(metric="Mreads/s (150 bp) edit Q20 trim + stats",
               unit="Mreads/s", reads=62_500_000, batch=12_500_000, L=150, seed=4,
               workload="C4: edit --left-length 10 --left-quality-range 20, --right-length 30 "
                        "--right-quality-range 20, + stats (500 M reads over 8 GPUs)"),
    "c5": dict(metric="Mreads/s (250 bp) chaos game k=7 tables",
               unit="Mreads/s", reads=25_000_000, batch=5_000_000, L=250, seed=5,
               workload="C5: chaos game k=7 feature tables (200 M x 250 bp over 8 GPUs)"),
    "c5_valid": dict(metric="Mreads/s (250 bp) chaos game k=7 tables, ONLY_VALID_READS",
                     unit="Mreads/s", reads=25_000_000, batch=5_000_000, L=250, seed=5,
                     workload="C5 with a read_status array marking a random 5 % of reads invalid "
                              "(ONLY_VALID_READS, old/chaos_game.c:188; the CLI's `stats --cg` with a filter)"),
    # routing / geometry cases, not BASELINE configs
    "c2_1024": dict(metric="Mreads/s (150 bp) stats+filter, lmax 1024 (drop-in default)",
                    unit="Mreads/s", reads=100_000_000, batch=10_000_000, L=150, seed=2, lmax=1024,
                    workload="C2 flags with the CLI's default --lmax 1024 (routing by read length)"),
    "c2_250": dict(metric="Mreads/s (250 bp) stats+filter",
                   unit="Mreads/s", reads=50_000_000, batch=5_000_000, L=250, seed=6,
                   workload="C2 flags on 250 bp reads (--lmax 250: wide geometry)"),
    "c2_250_1024": dict(metric="Mreads/s (250 bp) stats+filter, lmax 1024",
                        unit="Mreads/s", reads=50_000_000, batch=5_000_000, L=250, seed=6, lmax=1024,
                        workload="C2 flags on 250 bp reads with --lmax 1024 (hex defers to wide)"),
    # probes: C1 flags (stats, no filter) and a filter every read passes
    "c1_gpu": dict(metric="Mreads/s (150 bp) stats only", unit="Mreads/s", reads=100_000_000,
                   batch=10_000_000, L=150, seed=2, workload="C1 flags (stats, no filter) on the GPU"),
    "c2_nofail": dict(metric="Mreads/s (150 bp) stats + a filter every read passes", unit="Mreads/s",
                      reads=100_000_000, batch=10_000_000, L=150, seed=2,
                      workload="stats + --read-quality-range 0, --read-length-range 1, (no failures)"),
    "c3_nofail": dict(metric="Mpairs/s (2x150 bp) paired-end, a filter every pair passes", unit="Mpairs/s",
                      reads=100_000_000, batch=10_000_000, L=150, seed=3,
                      workload="PE 2x150 stats + --read-quality-range 0, --read-length-range 1, (no failures)"),
    "c2_noor": dict(metric="Mreads/s (150 bp) stats+filter with N / out-of-range limits",
                    unit="Mreads/s", reads=100_000_000, batch=10_000_000, L=150, seed=2,
                    workload="C2 flags + --max-N 2 --max-out-of-quality 20"),
    "c4_noor": dict(metric="Mreads/s (150 bp) edit Q20 trim + --max-N 2 + stats",
                    unit="Mreads/s", reads=62_500_000, batch=12_500_000, L=150, seed=4,
                    workload="C4 flags + --max-N 2 (the post-trim filter, src/edit_fastq.c:159-164)"),
    "c4_pe": dict(metric="Mpairs/s (2x150 bp) paired-end edit Q20 trim + stats",
                  unit="Mpairs/s", reads=50_000_000, batch=10_000_000, L=150, seed=4,
                  workload="C4 trims on paired-end 2x150 + --read-quality-range 20, "
                           "(pair kept iff both mates pass; old/main_hpg_fastq_old.c:728)"),
    "dropin": dict(metric="Mreads/s (150 bp) stats+filter through hpgq_run_host, 10,000-read host batches",
                   unit="Mreads/s", reads=4_000_000, batch=10_000, L=150, seed=2,
                   workload="INTEGRATION.md's fastq_stats_worker: AoS reads packed per 10,000-read batch into the "
                            "ctx's staging slot (hpgq_host_batch), hpgq_run_host without a mask, one hpgq_sync per "
                            "worker at the end, 2 worker threads with one ctx each (src/stats_options.c:21-22)"),
    "c2_kmers": dict(metric="Mreads/s (150 bp) stats --kmers 5-mer counts (passed reads of C2)",
                     unit="Mreads/s", reads=50_000_000, batch=10_000_000, L=150, seed=2,
                     workload="stats --kmers on C2 reads: 5-mers of the reads that pass "
                              "--read-quality-range 20, --read-length-range 50, (engine mask), per start position"),
    "c2_lr": dict(metric="Mreads/s (150 bp) stats+filter with a 5' window filter",
                  unit="Mreads/s", reads=100_000_000, batch=10_000_000, L=150, seed=2,
                  workload="C2 flags + --left-length 10 --left-quality-range 20,"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--reads", type=int, default=None, help="reads (pairs) per GPU")
    ap.add_argument("--batch-reads", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end CLI leg (C2)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-reads", type=int, default=None,
                    help="reads of the CPU baseline's sample (default 2 M; 400 k for CGR)")
    ap.add_argument("--lmax", type=int, default=None, help="override the config's lmax")
    ap.add_argument("--route", default=None,
                    help="A/B only: engine kernel route (hpgq_debug_set_route: auto, single, tri, hex, "
                         "wide, auto_fixed)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="launcher + read sharding on CPU: gloo ranks, no GPU, no kernels")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1,
                    help="tests only (with --launch-dry-run): this rank exits 2 before the rendezvous")
    ap.add_argument("--share-device", action="store_true",
                    help="functional test of N ranks on fewer GPUs (ranks share device LOCAL_RANK mod "
                         "count; RCCL over its socket transport): not a scaling measurement")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.steps < 1 or a.warmup < 0:
        ap.error("--steps must be >= 1 and --warmup >= 0")
    cfg = CONFIGS[a.config]
    a.reads = a.reads or cfg["reads"]
    a.batch_reads = a.batch_reads or cfg["batch"]
    a.read_length, a.seed = cfg["L"], cfg["seed"]
    if a.lmax:
        cfg["lmax"] = a.lmax
    return a


def params_for(cfg, L):
    lmax = CONFIGS[cfg].get("lmax", L)
    if cfg in ("c4", "c4_noor", "c4_pe"):
        extra = dict(max_N=2) if cfg == "c4_noor" else {}
        if cfg == "c4_pe":
            extra = dict(read_quality_range="20,")
        p = H.edit_params(lmax=lmax, stats=True, left_length=10, left_quality_range="20,",
                          right_length=30, right_quality_range="20,", **extra)
        p.paired = 1 if cfg == "c4_pe" else 0
        return p
    if cfg == "c1_gpu":
        return H.stats_params(lmax=lmax)
    if cfg in ("c2_nofail", "c3_nofail"):
        p = H.stats_params(lmax=lmax, read_quality_range="0,", read_length_range="1,")
        p.paired = 1 if cfg == "c3_nofail" else 0
        return p
    extra = dict(left_length=10, left_quality_range="20,") if cfg == "c2_lr" else {}
    if cfg == "c2_noor":
        extra = dict(max_N=2, max_out_of_quality=20)
    p = H.stats_params(lmax=lmax, read_quality_range="20,", read_length_range="50,", **extra)
    if cfg == "c3":
        p.paired = 1
    return p


# ---- CPU baseline: the oracle (C + OpenMP) on a bounded sample --------------
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def native_oracle():
    """The oracle rebuilt HERE with -O3 -march=native: the tree's
    liboracle.so is built portable (-march=x86-64-v2) in the build container,
    whose CPU is not the GPU box's.  Falls back to the portable build."""
    import subprocess
    import tempfile
    src = [os.path.join(ROOT, "oracle", f) for f in ("hpgq_oracle.c", "refarch.c")]
    tmp = tempfile.mkdtemp(prefix="hpgq_oracle_")
    out = os.path.join(tmp, "liboracle_native.so")
    cmd = ["gcc", "-O3", "-march=native", "-std=c99", "-fopenmp", "-pthread", "-fPIC", "-ffp-contract=off",
           "-shared", "-o", out, *src, "-lm"]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=120)
        lib = C.CDLL(out)
        build = "gcc -O3 -march=native -fopenmp (built on this host)"
    except (OSError, subprocess.SubprocessError):
        lib = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        build = "gcc -O3 -march=x86-64-v2 -fopenmp (portable)"
    # the loaded library stays mapped; its file and directory can go
    for f in (out, tmp):
        try:
            os.remove(f) if f == out else os.rmdir(f)
        except OSError:
            pass
    return lib, build


def cgroup_cpu_quota():
    """Cores' worth of CPU time this job may use (cgroup v2 cpu.max), or None
    when unlimited / unknown: the GPU box may cap a job below its visible cores."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def omp_threads(default):
    """This job's CPU share from OMP_NUM_THREADS (its first field: nested
    OpenMP lists such as '16,1' are valid), else `default`."""
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "").split(",")[0]))
    except ValueError:
        return default


def cpu_baseline(args, params):
    lib, build = native_oracle()
    lib.oracle_run.restype = C.c_int
    lib.oracle_run.argtypes = [C.POINTER(H.Params), C.POINTER(H.Batch), C.POINTER(H.Batch),
                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    lib.oracle_synth.argtypes = [C.POINTER(H.Synth), C.c_int64, C.c_int64, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
    lib.oracle_cgr_fill_batches.restype = C.c_int
    lib.oracle_cgr_fill_batches.argtypes = [C.c_int, C.c_int, C.POINTER(H.Batch), C.c_void_p, C.c_int,
                                            C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    ncores = len(os.sched_getaffinity(0))
    # the GPU box gives one GPU's job a share of the host's cores and says so in
    # OMP_NUM_THREADS (16 there); sched_getaffinity shows the whole host
    threads = max(1, min(omp_threads(ncores), ncores))
    L = args.read_length
    cgr = args.config in ("c5", "c5_valid")
    n = args.cpu_reads or (400_000 if cgr else 2_000_000)
    mates = 2 if params.paired else 1
    bufs = []
    for m in range(mates):
        s = H.Synth(args.seed, L, 5, 5, 1, 33, m)
        idx = np.zeros(n + 1, np.int32)
        seq = np.zeros(n * L, np.uint8)
        qual = np.zeros(n * L, np.uint8)
        lib.oracle_synth(C.byref(s), 0, n, seq.ctypes.data, qual.ctypes.data, idx.ctypes.data)
        bufs.append((seq, qual, idx))
    bs = [H.Batch(n, sq.ctypes.data, ql.ctypes.data, ix.ctypes.data) for sq, ql, ix in bufs]
    nt = [threads]
    if args.config == "c2_kmers":
        lib.oracle_kmers.argtypes = [C.POINTER(H.Batch), C.c_void_p, C.c_int, C.c_void_p]
        lib.oracle_kmers.restype = C.c_int
        by_pos = np.zeros(1024 * (L - 4), np.uint64)
        run = lambda p=None: lib.oracle_kmers(C.byref(bs[0]), None, L, by_pos.ctypes.data)  # noqa: E731
        what = "oracle_kmers (hpgq_oracle.c, one thread), every read"
        threads = 1
    elif cgr:
        # independent fill calls (one per batch of 20 k reads) spread over the threads
        nb = 20
        per = n // nb
        sub = (H.Batch * nb)()
        sq, ql, ix = bufs[0]
        for i in range(nb):
            sub[i] = H.Batch(per, sq.ctypes.data, ql.ctypes.data, ix[i * per:].ctypes.data)
        ts = np.zeros(128 * 128, np.uint32)
        tq = np.zeros(128 * 128, np.uint32)
        wc = np.zeros(1, np.uint32)
        valid = args.config == "c5_valid"
        status = read_status(n, args.seed)
        sp = (C.c_void_p * nb)(*[status.ctypes.data + i * per for i in range(nb)])
        run = lambda p=None: lib.oracle_cgr_fill_batches(  # noqa: E731
            7, 33, sub, sp if valid else None, 1 if valid else 0, nb, ts.ctypes.data,
            tq.ctypes.data, wc.ctypes.data, nt[0])
        what = (f"oracle_cgr_fill_batches (old/chaos_game.c restated), {nb} fill calls"
                + (", ONLY_VALID_READS with the same 5 % invalid status" if valid else ""))
    else:
        mask = np.zeros(n, np.uint8)
        trim = np.zeros(n * mates, np.uint32)

        def run(p=params):
            ctr = np.zeros(H.counters_len(p.lmax) * mates, np.uint64)
            return lib.oracle_run(C.byref(p), C.byref(bs[0]), C.byref(bs[1]) if mates == 2 else None,
                                  mask.ctypes.data, trim.ctypes.data, ctr.ctypes.data, nt[0])
        what = "oracle_run (hpgq_oracle.c)"

    def timed(p=None, budget=args.cpu_seconds):
        done, t0 = 0, time.perf_counter()
        while True:
            assert (run(p) if p is not None else run()) == 0
            done += n
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el
    done, el = timed()
    out = {"value": round(done / el / 1e6, 3), "unit": CONFIGS[args.config]["unit"],
           "cores": threads, "kind": "port", "cpu": cpu_model(), "cores_visible": ncores,
           "build": build}
    # one pass on one thread beside the threaded figure
    nt[0] = 1
    t1 = time.perf_counter()
    assert run() == 0
    el1 = time.perf_counter() - t1
    out["value_1thread"] = round(n / el1 / 1e6, 3)
    # the whole host, SURVEY §8d's "threads = nproc": every visible core for a
    # short run (context: the line's value above is this GPU's CPU share; the
    # job's cgroup quota, when the box sets one, is stated beside it)
    if args.config != "c2_kmers":
        nt[0] = ncores
        da, ea = timed(budget=max(1.0, args.cpu_seconds / 3))
        out["value_allcores"] = round(da / ea / 1e6, 3)
        out["cores_allcores"] = ncores
        out["cpu_quota_cores"] = cgroup_cpu_quota()
    nt[0] = threads
    c1 = ""
    if args.config == "c2":
        # BASELINE.json configs[0] (C1): `stats` (no filter) on 1 M x 150 SE reads, CPU
        p1 = H.stats_params(lmax=150)
        d1, e1 = timed(p1, budget=max(2.0, args.cpu_seconds / 3))
        out["c1_stats_mreads_s"] = round(d1 / e1 / 1e6, 3)
        c1 = (f"; c1_stats_mreads_s: C1 `stats` without filter, same reads, {d1 // n} passes "
              f"in {e1:.1f} s")
    if args.config == "c2":
        out["refarch"] = refarch_baseline(lib, params, bs[0], n, budget=max(2.0, args.cpu_seconds / 3))
    out["sample"] = (f"{n} synthetic {L} bp {'pairs' if mates == 2 else 'reads'} (seed "
                     f"{args.seed}, same generator and options), {done // n} passes in "
                     f"{el:.1f} s; {what}, {threads} OpenMP threads (this GPU's CPU share; "
                     f"{ncores} visible); value_1thread: one pass on 1 thread ({el1:.1f} s); "
                     f"value_allcores: the same on all {ncores} visible cores"
                     f"{allcores_note(out.get('cpu_quota_cores'), ncores)}{c1}")
    return out


def allcores_note(quota, ncores):
    """A cgroup CPU quota below the visible cores makes the all-core run
    time-share that many CPUs: say so beside the number."""
    if quota and quota < ncores:
        return (f" (the job's cgroup quota is {quota:g} CPUs, so the {ncores} threads time-share "
                f"them: the host's {ncores}-core rate is not measurable from this job)")
    return ""


def refarch_baseline(lib, params, batch, n, budget):
    """The reference's own stats architecture on the CPU (oracle/refarch.c):
    2 worker threads (src/stats_options.c:21) build per-read records per
    10,000-read batch (:22), ONE consumer merges them base by base through
    hash maps (src/stats_fastq.c:257-417).  Context beside the OpenMP port,
    never a target; timed on the first reads of the port's sample."""
    lib.refarch_stats.restype = C.c_int
    lib.refarch_stats.argtypes = [C.POINTER(H.Params), C.POINTER(H.Batch), C.c_int, C.c_int, C.c_void_p]
    m = min(n, 400_000)
    sub = H.Batch(m, batch.seq, batch.quality, batch.data_indices)
    ctr = np.zeros(H.counters_len(params.lmax), np.uint64)
    done, t0 = 0, time.perf_counter()
    while True:
        assert lib.refarch_stats(C.byref(params), C.byref(sub), 10_000, 2, ctr.ctypes.data) == 0
        done += m
        el = time.perf_counter() - t0
        if el >= budget:
            break
    return {"value": round(done / el / 1e6, 3), "unit": "Mreads/s", "cores": 3, "kind": "refarch",
            "sample": f"first {m} reads of the port's sample, {done // m} passes in {el:.1f} s: "
                      "oracle/refarch.c, 2 worker threads (10,000-read batches) + 1 hash-map "
                      "consumer thread, the shape of src/stats_fastq.c:202-417"}


def read_status(n, seed, first=0):
    """c5_valid's read_status[]: 1 (VALID_READ) except a random 5 % (0),
    counter-based per read index so any shard regenerates its slice."""
    i = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (i + np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) * np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(31)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(29)
    return ((x % np.uint64(100)) >= np.uint64(5)).astype(np.uint8)


# ---- end to end: FASTQ file -> the CLI (SURVEY §8d's second throughput) -----
E2E_READS = 20_000_000   # 6.2 GB of FASTQ text: a run of ~0.15 s, 25 chunks of 256 MB


def numa_cpus(device):
    """The CPUs of `device`'s NUMA node this process may use (empty: unknown)."""
    node = H.lib.hpgq_device_numa_node(device)
    if node < 0:
        return set()
    try:
        spec = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in spec.split(","):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus & os.sched_getaffinity(0)


def e2e_leg(args, device, runs=5, writer_runs=3):
    """`hpg-fastq stats --read-quality-range 20, --read-length-range 50,` on a
    synthetic FASTQ file in /dev/shm (tools/fqgen.c: the same generator,
    E2E_READS x 150 bp, written by threads on the GPU's NUMA node so the file's
    pages sit there), one warm-up run and `runs` back-to-back CLI runs on this
    one GPU; then the writing subcommands on the same file (`filter` with the
    same flags -> passed.fq + failed.fq, `edit` with C4's trims -> edit.fq), their
    outputs in /dev/shm too, `writer_runs` runs each.  The CLI's own throughput
    line (text read -> parse -> engine -> outputs written, its clock starting after
    device set-up) per run.  PCIe-inclusive: NOT the bench value."""
    import re
    import shutil
    import subprocess
    import tempfile
    cli = os.path.join(ROOT, "hpg-fastq_amd", "hpg-fastq")
    if not os.path.exists(cli):
        return {"error": "hpg-fastq not built"}
    tmp = tempfile.mkdtemp(prefix="hpgq_e2e_")
    gen = os.path.join(tmp, "fqgen")
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else tmp
    fq = os.path.join(shm, f"hpgq_e2e_{os.getpid()}.fq")
    outd = os.path.join(shm, f"hpgq_e2e_out_{os.getpid()}")
    cpus = numa_cpus(device)
    share = sorted(cpus)[:omp_threads(len(cpus) or 16)] if cpus else None
    nthr = str(len(share) if share else 16)
    out = {"reads": E2E_READS, "read_length": 150, "runs": runs,
           "command": "hpg-fastq stats -f <file> --read-quality-range 20, --read-length-range 50, "
                      f"--gpus 1 --num-threads {nthr}",
           "numa_cpus": len(share) if share else None}
    c2 = ["--read-quality-range", "20,", "--read-length-range", "50,"]
    c4 = ["--left-length", "10", "--left-quality-range", "20,", "--right-length", "30",
          "--right-quality-range", "20,"]

    def cli_runs(cmd, flags, n, warm, writers=None):
        vals, gbs = [], []
        for rep in range(n + (1 if warm else 0)):   # a warm-up run (GPU clocks, file pages): not counted
            shutil.rmtree(outd, ignore_errors=True)
            os.makedirs(outd)
            r = subprocess.run([cli, cmd, "-f", fq, "-o", outd, *flags, "--gpus", "1", "--gpu", str(device),
                                "--num-threads", nthr], check=True, capture_output=True, text=True, timeout=300)
            m = re.search(r"Throughput: (\d+) reads, ([0-9.]+) GB of FastQ in ([0-9.]+) s = ([0-9.]+) Mreads/s",
                          r.stdout)
            if not m:
                raise RuntimeError(f"{cmd}: no throughput line")
            if warm and rep == 0:
                continue
            w = re.search(r"Output writer\s*:\s*(.+)", r.stdout)
            if writers is not None and w:
                writers.add(w.group(1).strip())
            vals.append(float(m.group(4)))
            gbs.append(float(m.group(2)) / float(m.group(3)))
        return vals, gbs
    try:
        subprocess.run(["gcc", "-O2", "-fopenmp", os.path.join(ROOT, "tools", "fqgen.c"), "-o", gen],
                       check=True, capture_output=True, timeout=120)
        # fqgen pins itself to the GPU's NUMA CPUs (no preexec_fn: this process
        # may already run GPU runtime threads)
        subprocess.run([gen, fq, str(E2E_READS), "150", "2", ",".join(map(str, share or []))], check=True,
                       capture_output=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS=nthr))
        out["fastq_gb"] = round(os.path.getsize(fq) / 1e9, 3)
        vals, gbs = cli_runs("stats", c2, runs, True)
        out.update(mreads_s=round(float(np.median(vals)), 2), mreads_s_min=round(min(vals), 2),
                   mreads_s_runs=[round(v, 2) for v in vals], gb_s_fastq=round(float(np.median(gbs)), 2))
        for cmd, flags in (("filter", c2), ("edit", c4)):
            if writer_runs <= 0:
                break
            writers = set()
            vals, gbs = cli_runs(cmd, flags, writer_runs, False, writers)
            out[cmd] = {"writer": ", ".join(sorted(writers)) or None,"command": f"hpg-fastq {cmd} -f <file> -o /dev/shm/... {' '.join(flags)} --gpus 1 "
                                   f"--num-threads {nthr}",
                        "mreads_s": round(float(np.median(vals)), 2), "mreads_s_min": round(min(vals), 2),
                        "mreads_s_runs": [round(v, 2) for v in vals],
                        "gb_s_fastq": round(float(np.median(gbs)), 2)}
    except (OSError, subprocess.SubprocessError, RuntimeError) as e:
        out["error"] = str(e)[:200]
    finally:
        for f in (fq, gen):
            try:
                os.remove(f)
            except OSError:
                pass
        shutil.rmtree(outd, ignore_errors=True)
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def dropin_main(args):
    """--config dropin: INTEGRATION.md's stats worker (tools/dropin_bench.c) on
    10,000-read batches packed into the ctx's staging slot (hpgq_host_batch),
    2 worker threads with one ctx each, over a synthetic FASTQ file (reads
    loaded as AoS before the clock starts).  The value is the stats worker as
    the stats consumer needs it: no mask, no per-batch hpgq_sync, one sync per
    worker at the end (--no-sync).  Beside it: the worker that waits for each
    batch's mask (filter-style, hpgq_sync per batch) and the malloc'd-batch
    worker that hpgq_run_host copies."""
    import subprocess
    import tempfile
    harness = os.path.join(ROOT, "tools", "dropin_bench")
    tmp = tempfile.mkdtemp(prefix="hpgq_dropin_")
    gen = os.path.join(tmp, "fqgen")
    fq = os.path.join("/dev/shm" if os.path.isdir("/dev/shm") else tmp, f"hpgq_dropin_{os.getpid()}.fq")
    n = args.reads
    try:
        subprocess.run(["gcc", "-O2", "-fopenmp", os.path.join(ROOT, "tools", "fqgen.c"), "-o", gen],
                       check=True, capture_output=True, timeout=120)
        subprocess.run([gen, fq, str(n), "150", "2"], check=True, capture_output=True, timeout=300)
        base = [harness, fq, "--threads", "2", "--batch", str(args.batch_reads), "--c2",
                "--lmax", "1024", "--repeat", str(args.steps)]

        def harness_run(extra):
            r = subprocess.run(base + extra, check=True, capture_output=True, text=True, timeout=600)
            return json.loads(r.stdout.strip().splitlines()[-1])
        rec = harness_run(["--no-sync"])
        rec_sync = harness_run([])
        rec_copy = harness_run(["--copy"])
    finally:
        for f in (fq, gen):
            try:
                os.remove(f)
            except OSError:
                pass
        os.rmdir(tmp)
    cfg = CONFIGS["dropin"]
    out = {"metric": cfg["metric"], "value": rec["mreads_s"], "unit": cfg["unit"], "n_gpus": 1,
           "steps": args.steps, "warmup": 0, "ms_per_step": round(rec["best_s"] * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic FASTQ (tools/fqgen.c), host memory",
           "config": {"workload": cfg["workload"], "reads": rec["reads"], "batch_reads": rec["batch_reads"],
                      "threads": rec["threads"], "lmax": 1024, "staging": rec["staging"], "sync": rec["sync"]},
           "harness": rec,
           "sync_per_batch": {"mreads_s": rec_sync["mreads_s"], "mreads_s_mean": rec_sync["mreads_s_mean"],
                              "note": "the worker waits for each batch's mask (hpgq_sync per batch)"},
           "copy_path": {"mreads_s": rec_copy["mreads_s"], "mreads_s_mean": rec_copy["mreads_s_mean"],
                         "note": "worker packs into malloc'd buffers; hpgq_run_host copies them; sync per batch"}}
    print(json.dumps(out), flush=True)


# ---- resident synthetic shard ----------------------------------------------
def make_batches(args, rank, dev, mates):
    import torch
    L = args.read_length
    out = []   # per batch: (n, [(seq, qual, idx) per mate], alg bytes)
    first = rank * args.reads
    for lo in range(0, args.reads, args.batch_reads):
        n = min(args.batch_reads, args.reads - lo)
        per_mate = []
        nbytes = 0
        for m in range(mates):
            s = H.Synth(args.seed, L, 5, 5, 1, 33, m)
            idx = np.zeros(n + 1, np.int32)
            H.check(H.lib.hpgq_synth_indices_host(C.byref(s), first + lo, n, idx.ctypes.data),
                    "idx")
            nb = int(idx[-1])
            d_seq = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
            d_qual = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
            d_idx = torch.from_numpy(idx).to(dev)
            torch.cuda.synchronize()
            H.check(H.lib.hpgq_synth_device(C.byref(s), first + lo, n, d_seq.data_ptr(),
                                            d_qual.data_ptr(), d_idx.data_ptr(), None), "synth")
            torch.cuda.synchronize()
            per_mate.append((d_seq, d_qual, d_idx))
            nbytes += 2 * nb + 4 * (n + 1)   # seq + quality + 4-byte offsets
        out.append((n, per_mate, nbytes))
    return out


# ---- N ranks: the launcher (no GPU in this process) --------------------------
def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` (N > 1) without WORLD_SIZE: start N rank processes of this
    script, one per GPU (the old tool's --gpu-num-devices,
    old/main_hpg_fastq_old.c:113,161), with RANK / LOCAL_RANK / WORLD_SIZE and a
    127.0.0.1 rendezvous, and relay rank 0's JSON line.  This process never
    touches the GPU (nor loads libhpgq) and never execs: the ranks are fresh
    child interpreters.  A rank that fails ends the others; the exit code is
    the first failure's."""
    import subprocess
    n = args.gpus
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        if args.share_device:
            # ranks sharing one device: RCCL refuses two ranks on one GPU of one
            # host, so each rank names its own host and the ranks talk over
            # RCCL's socket transport on loopback (function, not speed)
            env.update(NCCL_HOSTID=f"hpgq-bench-rank{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    rc = 0
    while True:
        # (poll EVERY rank each time: `any(p.poll() is None ...)` stops at the
        # first running one and never sees a later rank that failed)
        states = [p.poll() for p in procs]
        if all(st is not None for st in states):
            break
        bad = [st for st in states if st not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t_end = time.time() + 15
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, t_end - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.1)
    out = procs[0].stdout.read()
    procs[0].stdout.close()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    if rc == 0 and line:
        print(line[-1], flush=True)
    elif rc == 0:
        print("bench: rank 0 printed no result line", file=sys.stderr)
        rc = 1
    return rc


def rank_fail(code, msg=None):
    """End a rank process now: os._exit, not sys.exit -- once libhpgq / HIP is
    loaded, interpreter teardown can block on runtime threads, and a rank that
    never exits leaves the others waiting at the rendezvous (the launcher only
    ends them when one has exited non-zero)."""
    if msg:
        print(msg, file=sys.stderr)
    sys.stderr.flush()
    sys.stdout.flush()
    os._exit(code)


def rank_env(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(`python bench.py --gpus N` starts them, or torch.distributed.run --nproc-per-node N)",
              file=sys.stderr)
        sys.exit(2)
    return world, rank, local


def shard(args, rank):
    """Rank r owns reads [r*R, (r+1)*R) of the counter-based generator."""
    return [rank * args.reads, (rank + 1) * args.reads]


def device_id(dev_index):
    """PCI address and UUID of a HIP device (torch's device properties)."""
    import torch
    pr = torch.cuda.get_device_properties(dev_index)
    pci = f"{getattr(pr, 'pci_domain_id', 0):04x}:{getattr(pr, 'pci_bus_id', 0):02x}:{getattr(pr, 'pci_device_id', 0):02x}"
    return pci, str(getattr(pr, "uuid", ""))


def rank_table(dist, world, mine):
    """N > 1: every rank's record (rank, device, PCI address, timed seconds,
    hot-kernel launch time) gathered on rank 0 over gloo, in rank order, so a
    slow or shared rank is visible in the one line."""
    got = [None] * world
    dist.all_gather_object(got, mine)
    return sorted(got, key=lambda g: g["rank"])


def check_distinct_devices(ranks, share_device):
    """Ranks on one node must hold distinct GPUs (one PCI function each) unless
    --share-device asks for the functional shared run; returns an error or None."""
    seen = {}
    for g in ranks:
        key = (g["pci"], g["uuid"])
        if key in seen and not share_device:
            return (f"bench: ranks {seen[key]} and {g['rank']} share device {g['pci']} "
                    f"(uuid {g['uuid']}); pass --share-device for a functional run")
        seen.setdefault(key, g["rank"])
    return None


def result_line(args, cfg, world, el, steps_reads, roofline, rccl_ranks, dtype, extra_config=None):
    cfgd = {"workload": cfg["workload"], "reads_per_gpu": args.reads, "read_length": args.read_length,
            "batch_reads": args.batch_reads,
            "parallelism": f"read-sharded x{world}, RCCL all-reduce of "
                           + ("the u32 CGR tables" if args.config in ("c5", "c5_valid") else "the counters")}
    if world > 1:
        cfgd["rccl_ranks"] = rccl_ranks
    cfgd.update(extra_config or {})
    return {
        "metric": cfg["metric"],
        "value": None if el is None else round(steps_reads / el / 1e6, 2),
        "unit": cfg["unit"],
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None if el is None else round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (counter-based generator, resident in HBM)",
        "config": cfgd,
        "roofline": roofline,
    }


RANK_KEYS = ("rank", "device", "pci", "uuid", "el_s", "avg_launch_us")


def dry_run_rank(args, world, rank):
    """--launch-dry-run: the rank plumbing on CPU.  Each rank derives its read
    range, fills the host offsets of its first reads with the same generator
    (hpgq_synth_indices_host: no device), and rank 0 checks over gloo that the
    ranges are disjoint and cover [0, world*R) before printing the line."""
    import torch.distributed as dist
    _load_hpgfastq()
    cfg = CONFIGS[args.config]
    if rank == args.dry_run_fail_rank:   # (the launcher must end the ranks left waiting)
        rank_fail(2, f"bench: rank {rank} fails (--dry-run-fail-rank)")
    if world > 1:
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        # (a bounded rendezvous: a peer that never arrives ends this rank too;
        # a fresh box's first `import torch` alone can take 1-2 minutes)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=900))
    lo, hi = shard(args, rank)
    n = min(1000, args.reads)
    s = H.Synth(args.seed, args.read_length, 5, 5, 1, 33, 0)
    idx = np.zeros(n + 1, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), lo, n, idx.ctypes.data), "idx")
    mine = {"rank": rank, "range": [lo, hi], "first_bytes": int(idx[-1]), "pid": os.getpid(),
            # the per-rank record of a real N > 1 line (no device here)
            "device": None, "pci": f"dry-run-{rank}", "uuid": "", "el_s": None, "avg_launch_us": None}
    t0 = time.perf_counter()
    got = [None] * world
    if world > 1:
        dist.all_gather_object(got, mine)
        dist.barrier()
    else:
        got = [mine]
    el = time.perf_counter() - t0
    if rank == 0:
        ranges = sorted(g["range"] for g in got)
        ok = ranges[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ranges, ranges[1:])) \
            and ranges[-1][1] == world * args.reads and len({g["pid"] for g in got}) == world
        if not ok:
            print(f"bench: bad shards {got}", file=sys.stderr)
            sys.exit(3)
        extra = {"dry_run": True, "shards": [g["range"] for g in sorted(got, key=lambda g: g["rank"])],
                 "rendezvous_s": round(el, 4)}
        if world > 1:
            extra["ranks"] = [{k: g[k] for k in RANK_KEYS} for g in sorted(got, key=lambda g: g["rank"])]
            err = check_distinct_devices(extra["ranks"], args.share_device)
            if err:
                print(err, file=sys.stderr)
                sys.exit(3)
        out = result_line(args, cfg, world, None, 0, None, None, "u8", extra)
        out["dry_run"] = True
        if world == 1 and not args.no_cpu_baseline:   # the CPU leg needs no device
            out["cpu_baseline"] = cpu_baseline(args, params_for(args.config, args.read_length))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world, rank, local = rank_env(args)
    if args.launch_dry_run:
        return dry_run_rank(args, world, rank)
    _load_hpgfastq()
    if args.config == "dropin":
        if world > 1:
            rank_fail(2, "bench: --config dropin is a one-GPU host-path harness")
        return dropin_main(args)
    cfg = CONFIGS[args.config]
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if local >= ndev and not args.share_device:
        rank_fail(2, f"bench: rank {rank} needs device {local} but {ndev} are visible")
    local_dev = local % max(ndev, 1)
    if world > 1:   # rank control on gloo; the data path's exchange is libhpgq's RCCL
        # one node: gloo on loopback (the container hostname may not resolve)
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        # (a bounded rendezvous: a peer that never arrives ends this rank too;
        # a fresh box's first `import torch` alone can take 1-2 minutes)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=900))
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:   # ranks on one GPU fail BEFORE RCCL init, warmup and timing
        pci, uuid = device_id(local_dev)
        err = check_distinct_devices(rank_table(dist, world, {"rank": rank, "pci": pci, "uuid": uuid}),
                                     args.share_device)
        if err:
            rank_fail(3, err if rank == 0 else None)

    L = args.read_length
    cgr = args.config in ("c5", "c5_valid")
    valid = args.config == "c5_valid"
    params = params_for(args.config, L)
    mates = 2 if params.paired else 1
    batches = make_batches(args, rank, dev, mates)
    d_mask = torch.empty(args.reads, dtype=torch.uint8, device=dev)
    d_trim = torch.empty(args.reads * mates, dtype=torch.int32, device=dev)
    offs = np.cumsum([0] + [b[0] for b in batches])

    statuses = []
    kmers = args.config == "c2_kmers"
    km = None
    if kmers:
        # the engine's C2 masks once (setup), then each step counts the passed
        # reads' 5-mers: the k-mer kernel alone is what the step times
        eng = H.Engine(params, device=local_dev)
        for i, (n, mm, _nb) in enumerate(batches):
            sq, ql, ix = mm[0]
            eng.run_device(H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr()), None,
                           d_mask.data_ptr() + int(offs[i]), None)
        eng.sync()
        km = H.Kmers(L, device=local_dev, stream=eng.stream)
        kernel_name = "hpgq::kmers::kmer_tile_kernel (+kmer_reduce_kernel; +kmer_maxlen_kernel above 8 tiles)"
        # seq + offsets + the mask (quality is not read)
        alg = [(nb - 4 * (n + 1)) // 2 + 4 * (n + 1) + n for (n, _m, nb) in batches]
    elif cgr:
        eng = H.ChaosGame(7, 33, device=local_dev)
        kernel_name = f"hpgq::cgr::stream::cgr_stream_kernel<7, {'true' if valid else 'false'}> (+span_first)"
        # algorithmic bytes per read: seq + quality + offset (tables stay in LDS)
        # (+ 1 status byte per read; the skipped reads' bytes are streamed too)
        alg = [nb + (n if valid else 0) for (n, _m, nb) in batches]
        if valid:
            lo = 0
            for (n, _m, _nb) in batches:
                statuses.append(torch.from_numpy(read_status(n, args.seed, rank * args.reads + lo)).to(dev))
                lo += n
            torch.cuda.synchronize()
    else:
        eng = H.Engine(params, device=local_dev, route=args.route)
        kernel_name = eng.kernel_name
        # + 1 B mask per read (pair), + 4 B trim per read when editing
        alg = [nb + n + (4 * n * mates if params.edit_on else 0) for (n, _m, nb) in batches]
    rccl_ranks = None
    if world > 1:   # one RCCL communicator inside libhpgq (counters / CGR tables)
        uid = H.engine.comm_unique_id() if rank == 0 else b"\0" * 128
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(world, rank, obj[0])
        rccl_ranks = eng.comm_count()
        if rccl_ranks != world:
            rank_fail(3, f"bench: RCCL communicator has {rccl_ranks} ranks, world is {world}")
    ext = torch.cuda.ExternalStream(eng.stream, device=dev)
    hb = [[H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr())
           for (sq, ql, ix) in mm] for (n, mm, _nb) in batches]
    # HIP events on the engine stream bracket the timed launches: ONE pair
    # around all K steps' launches (the steps queue back to back; an event pair
    # between two launches leaves a ~10 us gap, so none sit between launches),
    # or per step when the steps are separated by a host sync (CGR) or by the
    # RCCL all-reduce (N > 1), which the brackets leave out.
    # avg launch = bracketed GPU time / launches (it includes the chain's idle
    # follow-up stages and the resets: a slight overstatement of the kernel).
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    nb = len(hb)
    per_step = cgr or world > 1

    def step(s=None):
        (km if kmers else eng).reset()
        for i, b in enumerate(hb):
            if s is not None and i == 0 and (per_step or s == 0):
                ev[s][0].record(ext)
            if kmers:
                km.count_device(b[0], d_mask.data_ptr() + int(offs[i]))
            elif cgr:
                if valid:
                    eng.fill_device(b[0], statuses[i].data_ptr(), H.CGR_ONLY_VALID_READS)
                else:
                    eng.fill_device(b[0])
            else:
                eng.run_device(b[0], b[1] if mates == 2 else None,
                               d_mask.data_ptr() + int(offs[i]),
                               d_trim.data_ptr() + 4 * int(offs[i]) if params.edit_on else None)
            if s is not None and i == nb - 1 and (per_step or s == args.steps - 1):
                ev[s][1].record(ext)
        if world > 1 and not kmers:   # the one exchange step: RCCL sum of the counters / u32 CGR tables
            eng.allreduce()

    for _ in range(args.warmup):
        step()
    eng.sync()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(s)
        if cgr:   # a gated CGR call is redone exactly inside the sync: once per step
            eng.sync()
    # the engine steps queue back to back on the stream (stream-ordered resets);
    # one host sync after the K steps (it also returns the error flag)
    eng.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if per_step:
        timed_ms = sum(a.elapsed_time(b) for a, b in ev)
    else:
        timed_ms = ev[0][0].elapsed_time(ev[-1][1])
    ranks = None
    if world > 1:
        # every rank's own clock and hot-kernel time, then the max over ranks
        pci, uuid = device_id(local_dev)
        ranks = rank_table(dist, world, {"rank": rank, "device": local_dev, "pci": pci, "uuid": uuid,
                                         "el_s": round(el, 6),
                                         "avg_launch_us": round(timed_ms / (args.steps * nb) * 1e3, 1)})
        el = max(g["el_s"] for g in ranks)

    # sanity: every read accounted for (after the all-reduce: every rank's reads)
    if kmers:
        assert int(km.by_pos().sum()) > 0 or os.environ.get("HPGQ_BENCH_NOCHECK")   # (timing probes)
    elif cgr:
        _ts, _tq, wc = eng.tables()
        assert wc > 0 or os.environ.get("HPGQ_BENCH_NOCHECK")   # (timing-probe builds add nothing)
    else:
        ctr = eng.counters()
        expect = args.reads * world
        assert int(ctr[H.S_NUM_INPUT]) == expect, (int(ctr[H.S_NUM_INPUT]), expect)

    total = args.reads * world * args.steps
    avg_launch_s = timed_ms / (args.steps * nb) / 1e3
    bytes_per_launch = float(np.mean(alg))
    achieved = bytes_per_launch / avg_launch_s / 1e9

    # HBM bytes per launch: NOT measured in this run (PMC counters need their
    # own rocprofv3 passes); taken from the committed PMC profile of the same
    # kernel and batch size, and labelled with its file
    traffic, traffic_src = None, None
    pmc_rel = os.path.join("profiles", f"pmc_engine_{args.config}.json")
    pmc = os.path.join(ROOT, pmc_rel)
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))
            if rec.get("kernel") == kernel_name and rec.get("batch_reads") == args.batch_reads:
                traffic = rec.get("hbm_bytes_per_launch")
                traffic_src = pmc_rel + " (committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes, not this run)"
        except (OSError, ValueError):
            traffic = None

    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": traffic_src, "kernel": kernel_name,
                "avg_launch_us": round(avg_launch_s * 1e6, 1),
                "alg_bytes_per_launch": int(bytes_per_launch)}
    extra = {"route": args.route} if args.route else {}
    if ranks is not None:
        extra["ranks"] = ranks
    else:   # which GPU ran it: profiles are checked against this line's clock (tools/profile_report.py)
        pci, uuid = device_id(local_dev)
        extra["device"] = {"index": local_dev, "pci": pci, "uuid": uuid}
    if args.share_device:
        extra["shared_device"] = f"{world} ranks on {ndev} device(s): functional run, not a scaling number"
    out = result_line(args, cfg, world, el, total, roofline, rccl_ranks, "f64" if cgr else "u8", extra)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, params)
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_e2e:
        eng.close()   # (the CLI runs in its own process)
        eng = None
        out["e2e"] = e2e_leg(args, local_dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if km is not None:
        km.close()
    if eng is not None:
        eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
