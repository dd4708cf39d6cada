"""Profiling driver: the C2 engine kernel on one resident 10M-read batch.

Run under rocprofv3 (kernel trace or --pmc passes); no timing of its own.
  python tools/prof_engine.py [--reads N] [--iters K] [--mode c2|stats|edit|edit0|editL|editR|maxn|pe|cgr|cgrv]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hpg-fastq_amd"))
import torch  # noqa: E402  (device buffers; imported before hpgfastq: one HIP runtime)
import hpgfastq as H  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, default=10_000_000)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--mode", default="c2")
ap.add_argument("--L", type=int, default=150)
ap.add_argument("--k", type=int, default=7)
ap.add_argument("--kmers", action="store_true", help="also count 5-mers (stats --kmers) after the engine")
ap.add_argument("--invalid-pct", type=float, default=None, help="cgrv: this share of skipped reads instead of bench.py's 5 %%")
args = ap.parse_args()

dev = torch.device("cuda", 0)
n, L = args.reads, args.L
if args.mode in ("cgr", "cgrv"):
    s = H.Synth(5, L, 5, 5, 1, 33, 0)
    idx = np.zeros(n + 1, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), 0, n, idx.ctypes.data), "idx")
    nb = int(idx[-1])
    sq = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
    ql = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
    ix = torch.from_numpy(idx).to(dev)
    torch.cuda.synchronize()
    H.check(H.lib.hpgq_synth_device(C.byref(s), 0, n, sq.data_ptr(), ql.data_ptr(),
                                    ix.data_ptr(), None), "synth")
    torch.cuda.synchronize()
    cg = H.ChaosGame(args.k)
    b = H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr())
    st = None
    if args.mode == "cgrv":   # ONLY_VALID_READS with bench.py's 5 % invalid status
        sys.path.insert(0, ROOT)
        from bench import read_status
        st = read_status(n, 5)
        if args.invalid_pct is not None:   # probes: another share of skipped reads (0: none)
            st = (np.random.default_rng(5).random(n) >= args.invalid_pct / 100).astype(np.uint8)
        st = torch.from_numpy(st).to(dev)
        torch.cuda.synchronize()
    for _ in range(args.iters):
        if st is not None:
            cg.fill_device(b, st.data_ptr(), H.CGR_ONLY_VALID_READS)
        else:
            cg.fill_device(b)
    cg.sync()
    print("cgr reads", n, "replays", cg.last_replays(), "words", cg.tables()[2])
    cg.close()
    sys.exit(0)
if args.mode == "c2":
    p = H.stats_params(lmax=L, read_quality_range="20,", read_length_range="50,")
elif args.mode == "lr":   # C2 plus a 5' window filter (the window-scan variant)
    p = H.stats_params(lmax=L, read_quality_range="20,", read_length_range="50,", left_length=10,
                       left_quality_range="20,")
elif args.mode == "nofail":   # a filter every read passes (no failed-read subtraction)
    p = H.stats_params(lmax=L, read_quality_range="0,", read_length_range="1,")
elif args.mode == "stats":
    p = H.stats_params(lmax=L)
elif args.mode == "edit":
    p = H.edit_params(lmax=L, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,")
elif args.mode == "maxn":   # C2 plus max_N / max_out_of_quality (the N / out-of-range filter variant)
    p = H.stats_params(lmax=L, read_quality_range="20,", read_length_range="50,", max_N=2,
                       max_out_of_quality=20)
elif args.mode == "pe_edit":   # C4 trims on paired-end (bench --config c4_pe)
    p = H.edit_params(lmax=L, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", read_quality_range="20,")
    p.paired = 1
elif args.mode == "edit_noor":   # C4 + --max-N 2 (bench --config c4_noor)
    p = H.edit_params(lmax=L, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", max_N=2)
elif args.mode in ("edit0", "editL", "editR"):   # timing probes: the edit kernel, fewer trims
    p = H.edit_params(lmax=L, stats=True, left_length=10 if args.mode == "editL" else 0,
                      left_quality_range="20,", right_length=30 if args.mode == "editR" else 0,
                      right_quality_range="20,")
else:
    p = H.stats_params(lmax=L, read_quality_range="20,", read_length_range="50,")
    p.paired = 1
nm = 2 if p.paired else 1
bufs = []
for m in range(nm):
    s = H.Synth(2, L, 5, 5, 1, 33, m)
    idx = np.zeros(n + 1, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), 0, n, idx.ctypes.data), "idx")
    nb = int(idx[-1])
    sq = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
    ql = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
    ix = torch.from_numpy(idx).to(dev)
    torch.cuda.synchronize()
    H.check(H.lib.hpgq_synth_device(C.byref(s), 0, n, sq.data_ptr(), ql.data_ptr(),
                                    ix.data_ptr(), None), "synth")
    torch.cuda.synchronize()
    bufs.append((sq, ql, ix))
mask = torch.empty(n, dtype=torch.uint8, device=dev)
trim = torch.empty(n * nm, dtype=torch.int32, device=dev)
eng = H.Engine(p)
bs = [H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr()) for sq, ql, ix in bufs]
for _ in range(args.iters):
    eng.run_device(bs[0], bs[1] if nm == 2 else None, mask.data_ptr(),
                   trim.data_ptr() if p.edit_on else None)
eng.sync()
c = eng.counters()
print("reads", n, "passed", int(c[H.S_NUM_PASSED]), "iters", args.iters)
if args.kmers:   # then --kmers counts of the passed reads (the engine's mask), args.iters times
    km = H.Kmers(L, stream=eng.stream)
    for _ in range(args.iters):
        km.count_device(bs[0], mask.data_ptr())
    km.sync()
    print("kmers", int(km.by_pos().sum()))
    km.close()
eng.close()
