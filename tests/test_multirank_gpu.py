"""libhpgq's RCCL path with more than one rank, on the one-GPU test box.

RCCL refuses two ranks on one GPU of one host ("Duplicate GPU detected"), so
each rank process names its own host (NCCL_HOSTID) and the ranks talk over
RCCL's socket transport on loopback.  That runs the real communicator set-up
(hpgq_comm_init / hpgq_cgr_comm_init with nranks 2), ncclCommCount and the
collectives (hpgq_allreduce, hpgq_cgr_allreduce) end to end; only the
transport differs from an 8-GPU node's xGMI.  Expected values: the oracle over
every rank's reads (counters: u64 sums; CGR: one fill call per CB reads per
rank, u32 sums).  Then bench.py's own launcher: `--gpus 2` starts two ranks.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
import rccl_rank

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
WORLD = 2


def _rank_env(r):
    return dict(os.environ, NCCL_HOSTID=f"hpgq-test-rank{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                HSA_ENABLE_IPC_MODE_LEGACY="0")


def _run_ranks(tmp_path):
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "rccl_rank.py"), str(r), str(WORLD),
                               str(tmp_path)], env=_rank_env(r), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True)
             for r in range(WORLD)]
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=150)
            logs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} rc={p.returncode}\n{logs[r][-3000:] if r < len(logs) else ''}"
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(WORLD)]


def test_rccl_two_ranks_counters_and_tables(tmp_path):
    res = _run_ranks(tmp_path)
    R = rccl_rank.R
    for name, p in zip(("c2", "c4"), rccl_rank.params()):
        want = np.zeros(H.counters_len(p.lmax), np.uint64)
        for r in range(WORLD):
            reads = O.synth(R, seed=2, L=150, first=r * R)
            m_o, t_o, c_o = O.run(p, reads)
            # each rank's own counters, masks and trims: the oracle on its shard
            np.testing.assert_array_equal(res[r][name + "_own"], c_o)
            half = R // 2
            for lo, hi in ((0, half), (half, R)):
                np.testing.assert_array_equal(res[r][f"{name}_mask_{lo}"], m_o[lo:hi])
                if p.edit_on:
                    np.testing.assert_array_equal(res[r][f"{name}_trim_{lo}"], t_o[lo:hi])
            want += c_o
        for r in range(WORLD):
            assert int(res[r][name + "_ranks"]) == WORLD
            # the all-reduced sum (twice: out of place, no double count)
            np.testing.assert_array_equal(res[r][name + "_sum"], want)
        assert int(want[H.S_NUM_INPUT]) == WORLD * R
    # the long-read ctx: each rank's own full-length set, and the collective
    # full-length sum at the longest read of ANY rank
    p = H.stats_params(lmax=150)
    Lg = max(max(v) for v in rccl_rank.LONG.values())
    want_dense = np.zeros(H.counters_len(150), np.uint64)
    want_ext = np.zeros(H.counters_len(Lg), np.uint64)
    for r in range(WORLD):
        lr = rccl_rank.long_reads(r)
        want_dense += O.run(p, lr)[2]
        Lr = max(rccl_rank.LONG[r])
        assert list(res[r]["lr_L"]) == [Lr, Lg]
        px = H.Params.from_buffer_copy(p)
        px.lmax = Lr
        np.testing.assert_array_equal(res[r]["lr_own_ext"], O.run(px, lr)[2])
        px.lmax = Lg
        want_ext += O.run(px, lr)[2]
    for r in range(WORLD):
        np.testing.assert_array_equal(res[r]["lr_sum"], want_dense)
        np.testing.assert_array_equal(res[r]["lr_sum_ext"], want_ext)
    dim2 = 128 * 128
    tables = (np.zeros(dim2, np.uint32), np.zeros(dim2, np.uint32), np.zeros(1, np.uint32))
    for r in range(WORLD):
        reads = O.synth(R, seed=2, L=150, first=r * R)
        for lo in range(0, R, rccl_rank.CB):
            hi = min(R, lo + rccl_rank.CB)
            a, b = int(reads.idx[lo]), int(reads.idx[hi])
            part = O.Reads(reads.seq[a:b].copy(), reads.qual[a:b].copy(),
                           (reads.idx[lo:hi + 1] - a).astype(np.int32))
            O.cgr(7, part, 33, tables=tables)
    for r in range(WORLD):
        assert int(res[r]["cgr_ranks"]) == WORLD
        np.testing.assert_array_equal(res[r]["cgr_ts"], tables[0])
        np.testing.assert_array_equal(res[r]["cgr_tq"], tables[1])
        assert int(res[r]["cgr_wc"][0]) == int(tables[2][0])


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_launches_two_ranks(config):
    """`python bench.py --gpus 2` starts two rank processes (here sharing the
    box's one GPU) whose RCCL communicator holds 2 ranks; bench asserts that
    the all-reduced counters hold both ranks' reads."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--config", config, "--reads", "2000000", "--batch-reads", "1000000", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert line["config"]["rccl_ranks"] == 2
    assert "shared_device" in line["config"]
    assert line["value"] > 0
    ranks = line["config"]["ranks"]   # per-rank clock, kernel time and device
    assert [g["rank"] for g in ranks] == [0, 1]
    assert all(g["el_s"] > 0 and g["avg_launch_us"] > 0 and g["pci"] for g in ranks)
    assert max(g["el_s"] for g in ranks) * 1e3 / 2 == pytest.approx(line["ms_per_step"], rel=1e-3, abs=1e-3)
