#!/usr/bin/env python3
"""bench.py — hpg-fastq hot path on MI355X: stats+filter Mreads/s.

Workload (BASELINE.json configs[1]): `hpg-fastq stats
--read-quality-range 20, --read-length-range 50,` over 100 M synthetic 150 bp
single-end reads PER GPU, resident in HBM (10 batches of 10 M reads, the
reference's fastq_batch_t layout).  One step = reset counters + the fused
edit->filter->stats kernel over every batch (+ one RCCL all-reduce of the
packed counters when N > 1).  Reads shard by index across ranks with no
data-path collective: weak scaling.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0) with `roofline` (engine kernel, HIP events on
the engine's own stream) and `cpu_baseline` (oracle/liboracle.so, C+OpenMP,
timed on this host's cores on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hpg-fastq_amd"))

import hpgfastq as H  # noqa: E402

METRIC = "Mreads/s (150 bp) stats+filter at 1/2/4/8 MI355X; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
FILTER_FLAGS = dict(read_quality_range="20,", read_length_range="50,")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=100_000_000, help="reads per GPU")
    ap.add_argument("--batch-reads", type=int, default=10_000_000)
    ap.add_argument("--read-length", type=int, default=150)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


def cpu_baseline(args, params):
    """Oracle (C + OpenMP) on a bounded sample of the same workload."""
    lib = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    lib.oracle_run.restype = C.c_int
    lib.oracle_run.argtypes = [C.POINTER(H.Params), C.POINTER(H.Batch), C.POINTER(H.Batch),
                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    lib.oracle_synth.argtypes = [C.POINTER(H.Synth), C.c_int64, C.c_int64, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
    ncores = len(os.sched_getaffinity(0))
    threads = max(1, min(16, ncores))
    n = 2_000_000
    s = H.Synth(args.seed, args.read_length, 5, 5, 1, 33, 0)
    idx = np.zeros(n + 1, np.int32)
    seq = np.zeros(n * args.read_length, np.uint8)
    qual = np.zeros(n * args.read_length, np.uint8)
    lib.oracle_synth(C.byref(s), 0, n, seq.ctypes.data, qual.ctypes.data, idx.ctypes.data)
    b = H.Batch(n, seq.ctypes.data, qual.ctypes.data, idx.ctypes.data)
    mask = np.zeros(n, np.uint8)
    ctr = np.zeros(H.counters_len(params.lmax), np.uint64)
    done, t0 = 0, time.perf_counter()
    while True:
        rc = lib.oracle_run(C.byref(params), C.byref(b), None, mask.ctypes.data, None,
                            ctr.ctypes.data, threads)
        assert rc == 0
        done += n
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    return {"value": round(done / el / 1e6, 3), "unit": "Mreads/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} synthetic {args.read_length} bp reads (seed {args.seed}, same "
                      f"generator and filter), {done // n} passes in {el:.1f} s; "
                      f"oracle/hpgq_oracle.c -O3 OpenMP, {threads} threads of {ncores} visible"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    L = args.read_length
    params = H.stats_params(lmax=L, **FILTER_FLAGS)
    eng = H.Engine(params, device=local)
    if world > 1:
        uid = H.engine.comm_unique_id() if rank == 0 else b"\0" * 128
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(world, rank, obj[0])

    # ---- resident synthetic shard: reads [rank*R, (rank+1)*R) -------------
    stream_ptr = eng.stream
    ext = torch.cuda.ExternalStream(stream_ptr, device=dev)
    batches = []
    total_bytes_alg = 0
    first = rank * args.reads
    s = H.Synth(args.seed, L, 5, 5, 1, 33, 0)
    for lo in range(0, args.reads, args.batch_reads):
        n = min(args.batch_reads, args.reads - lo)
        idx = np.zeros(n + 1, np.int32)
        H.check(H.lib.hpgq_synth_indices_host(C.byref(s), first + lo, n, idx.ctypes.data), "idx")
        nb = int(idx[-1])
        d_seq = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
        d_qual = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
        d_idx = torch.from_numpy(idx).to(dev)
        torch.cuda.synchronize()
        H.check(H.lib.hpgq_synth_device(C.byref(s), first + lo, n, d_seq.data_ptr(),
                                        d_qual.data_ptr(), d_idx.data_ptr(), None), "synth")
        torch.cuda.synchronize()
        batches.append((n, d_seq, d_qual, d_idx))
        # algorithmic bytes: seq + quality + 4-byte offset per read, 1-byte mask out
        total_bytes_alg += 2 * nb + 4 * (n + 1) + n
    d_mask = torch.empty(args.reads, dtype=torch.uint8, device=dev)
    hb = [H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr())
          for (n, sq, ql, ix) in batches]
    offs = np.cumsum([0] + [n for (n, *_r) in batches])

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in batches]

    def step(timed_events):
        eng.reset()
        for i, b in enumerate(hb):
            if timed_events:
                ev[i][0].record(ext)
            eng.run_device(b, None, d_mask.data_ptr() + int(offs[i]), None)
            if timed_events:
                ev[i][1].record(ext)
        if world > 1:
            eng.allreduce()

    for _ in range(args.warmup):
        step(False)
    eng.sync()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kern_ms = []
    for _ in range(args.steps):
        step(True)
        eng.sync()
        kern_ms.extend(a.elapsed_time(b) for a, b in ev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())

    # correctness sanity: every read accounted for in the final counters
    ctr = eng.counters()
    expect = args.reads * (world if world > 1 else 1)
    assert int(ctr[H.S_NUM_INPUT]) == expect, (int(ctr[H.S_NUM_INPUT]), expect)

    total_reads = args.reads * world * args.steps
    value = total_reads / el / 1e6
    avg_launch_s = float(np.mean(kern_ms)) / 1e3
    bytes_per_launch = total_bytes_alg / len(batches)
    achieved = bytes_per_launch / avg_launch_s / 1e9

    traffic = None
    # HBM bytes per launch from the committed PMC passes of the same kernel and
    # batch (tools/gpu_profile.sh -> tools/profile_report.py); only used when
    # they were taken on the kernel this run launched
    pmc = os.path.join(ROOT, "profiles", "pmc_engine_c2.json")
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))
            if rec.get("kernel") == eng.kernel_name and rec.get("batch_reads") == args.batch_reads:
                traffic = rec.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mreads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based generator, resident in HBM)",
        "config": {"workload": "C2: stats+filter --read-quality-range 20, --read-length-range 50,",
                   "reads_per_gpu": args.reads, "read_length": L, "batch_reads": args.batch_reads,
                   "parallelism": f"read-sharded x{world}, RCCL all-reduce of counters"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": eng.kernel_name,
                     "avg_launch_us": round(avg_launch_s * 1e6, 1),
                     "alg_bytes_per_launch": int(bytes_per_launch)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, params)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
