"""One rank of the multi-rank RCCL test (tests/test_multirank_gpu.py); run as a
script, one process per rank:  python rccl_rank.py RANK WORLD OUTDIR

Rank r owns reads [r*R, (r+1)*R) of the counter-based generator (bench.py's
sharding) and runs them through libhpgq only: the C2 stats+filter ctx and the
C4 edit+stats ctx (host path) and the chaos-game k = 7 ctx (one fill call per
CB reads, device batches), each with its own RCCL communicator
(hpgq_comm_init / hpgq_cgr_comm_init), then the libhpgq all-reduces
(hpgq_allreduce, hpgq_cgr_allreduce).  The reduced counters and tables are
saved for the test to compare with the oracle over all ranks' reads.  Rank 0
makes the unique ids and hands them over in a file (no other channel).
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "hpg-fastq_amd"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hpgfastq as H  # noqa: E402
import oracle_lib as O  # noqa: E402  (input generator only: O.synth)

R = 20000   # reads per rank
CB = 5000   # reads per chaos-game fill call
LONG = {0: [300, 3000], 1: [151, 9000, 700]}   # the long-read ctx's long reads per rank


def long_reads(rank):
    """Rank r's shard for the long-read ctx: 2,000 synthetic 150 bp reads with
    LONG[r] appended (each rank's longest read differs: the ranks must agree on
    lmax_ext in hpgq_read_counters_ext)."""
    base = O.synth(2000, seed=5, L=150, first=rank * 2000)
    rng = np.random.default_rng(100 + rank)
    extra = [(bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), L).astype(np.uint8)),
              bytes((33 + rng.integers(2, 42, L)).astype(np.uint8))) for L in LONG[rank]]
    return O.Reads.from_pairs(base.pairs() + extra)


def params():
    c2 = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    c4 = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                       right_length=30, right_quality_range="20,")
    return c2, c4


def uids(rank, outdir):
    path = os.path.join(outdir, "uids")
    if rank == 0:
        ids = b"".join(H.engine.comm_unique_id() for _ in range(4))
        with open(path + ".tmp", "wb") as f:
            f.write(ids)
        os.rename(path + ".tmp", path)
    t_end = time.time() + 60
    while not os.path.exists(path):
        if time.time() > t_end:
            raise SystemExit("rank %d: no unique ids from rank 0" % rank)
        time.sleep(0.05)
    ids = open(path, "rb").read()
    return [ids[i * 128:(i + 1) * 128] for i in range(4)]


def main():
    rank, world, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    ids = uids(rank, outdir)
    reads = O.synth(R, seed=2, L=150, first=rank * R)
    out = {}
    for name, p, uid in zip(("c2", "c4"), params(), ids[:2]):
        with H.Engine(p) as e:
            e.comm_init(world, rank, uid)
            out[name + "_ranks"] = e.comm_count()
            # two host batches, the all-reduce, one more all-reduce (out of place:
            # must not double count)
            half = R // 2
            for lo, hi in ((0, half), (half, R)):
                b = H.engine.host_batch(reads.seq, reads.qual, reads.idx[lo:hi + 1].copy())
                mask = np.zeros(hi - lo, np.uint8)
                trim = np.zeros(hi - lo, np.uint32)
                e.run_host(b, None, mask, trim if p.edit_on else None)
                e.sync()
                out[f"{name}_mask_{lo}"] = mask
                out[f"{name}_trim_{lo}"] = trim
            out[name + "_own"] = e.counters()
            e.allreduce()
            e.allreduce()
            out[name + "_sum"] = e.counters()
    # reads longer than lmax on both ranks: the full-length counters after the
    # all-reduce (hpgq_read_counters_ext, collective: both ranks call it)
    lr = long_reads(rank)
    with H.Engine(H.stats_params(lmax=150)) as e:
        e.comm_init(world, rank, ids[3])
        e.process(lr.seq, lr.qual, lr.idx)
        out["lr_own_ext"], L = e.counters_ext()
        e.allreduce()
        out["lr_sum"] = e.counters()
        out["lr_sum_ext"], Lg = e.counters_ext()
        out["lr_L"] = np.array([L, Lg])
    cg = H.ChaosGame(7, 33)
    cg.comm_init(world, rank, ids[2])
    out["cgr_ranks"] = cg.comm_count()
    dev = torch.device("cuda", 0)
    pad = np.zeros(H.DEVICE_SLACK, np.uint8)
    keep = []
    for lo in range(0, R, CB):
        hi = min(R, lo + CB)
        a, b = int(reads.idx[lo]), int(reads.idx[hi])
        seq = torch.from_numpy(np.concatenate([reads.seq[a:b], pad])).to(dev)
        qual = torch.from_numpy(np.concatenate([reads.qual[a:b], pad])).to(dev)
        idx = torch.from_numpy((reads.idx[lo:hi + 1] - a).astype(np.int32)).to(dev)
        torch.cuda.synchronize()
        keep.append((seq, qual, idx))
        cg.fill_device(H.engine.device_batch(hi - lo, seq.data_ptr(), qual.data_ptr(), idx.data_ptr()))
        cg.sync()
    cg.allreduce()
    ts, tq, wc = cg.tables()
    out.update(cgr_ts=ts.reshape(-1), cgr_tq=tq.reshape(-1), cgr_wc=np.array([wc], np.uint32))
    cg.close()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **{k: np.asarray(v) for k, v in out.items()})
    print(f"rank {rank}: done", flush=True)


if __name__ == "__main__":
    main()
