"""Multi-rank path on CPU (gloo, world_size 2): reads shard by index with no
data-path exchange (bench.py: rank r owns reads [r*R, (r+1)*R) of the
counter-based generator) and ONE sum all-reduce of the packed u64 counters
gives the single-process result.  The GPU path does the same reduction with
RCCL inside libhpgq (hpgq_allreduce); this checks the sharding and the
reduction's algebra with the oracle as the per-rank worker.  The same for the
chaos-game tables (hpgq_cgr_allreduce): each rank makes one fill call per
batch of its shard, and the u32 sum over ranks (int32 all-reduce: the same
bits) equals one process making every call."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

R = 3000   # reads per rank
CB = 500   # reads per CGR fill call (one call = one batch, old/chaos_game.c:165)


def _params():
    import hpgfastq as H
    return H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "hpg-fastq_amd"), here]
    import oracle_lib as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    reads = O.synth(R, seed=2, L=150, first=rank * R)
    _, _, ctr = O.run(_params(), reads, nthreads=1)
    t = torch.from_numpy(ctr.view(np.int64).copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    tables = _cgr_calls(O, reads)
    tc = torch.from_numpy(np.concatenate(tables).view(np.int32).copy())
    dist.all_reduce(tc, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out, t.numpy().view(np.uint64))
        np.save(out + ".cgr.npy", tc.numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


def _cgr_calls(O, reads, k=5):
    """One oracle chaos_game_fill_tables call per CB-read batch, summed (u32)."""
    dim = 1 << k
    tables = (np.zeros(dim * dim, np.uint32), np.zeros(dim * dim, np.uint32), np.zeros(1, np.uint32))
    for a in range(0, reads.n, CB):
        sub = O.Reads.from_pairs([reads.read(i) for i in range(a, min(a + CB, reads.n))])
        O.cgr(k, sub, 33, tables=tables)
    return tables


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_rank_shards_reduce_to_single_run(tmp_path):
    import oracle_lib as O
    out = str(tmp_path / "ctr.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    reduced = np.load(out)
    whole = O.synth(2 * R, seed=2, L=150, first=0)
    _, _, ctr = O.run(_params(), whole, nthreads=1)
    np.testing.assert_array_equal(reduced, ctr)
    np.testing.assert_array_equal(np.load(out + ".cgr.npy"), np.concatenate(_cgr_calls(O, whole)))
