"""bench.py's N-rank launcher on CPU (no GPU): `--gpus N` starts N rank
processes itself when WORLD_SIZE is unset, the ranks rendezvous on gloo at
127.0.0.1, each takes reads [r*R, (r+1)*R), and rank 0 prints ONE line with
n_gpus = N.  A --gpus / WORLD_SIZE mismatch exits non-zero."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")

# the keys of the driver's line (shape shared by the dry run and a real run)
LINE_KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
             "scaling", "vs_baseline", "dtype", "data", "config", "roofline"}


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _bench(*args, env=None):
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=240,
                          env=env or _env())


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_ranks_and_shards_reads(n):
    r = _bench("--gpus", str(n), "--launch-dry-run", "--reads", "5000", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout           # one line: rank 0's, relayed
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert set(line) - {"dry_run"} == LINE_KEYS
    assert line["config"]["shards"] == [[k * 5000, (k + 1) * 5000] for k in range(n)]
    # the per-rank diagnostics of an N > 1 line: one record
    # per rank in rank order with its device, PCI address, clock and kernel time
    ranks = line["config"]["ranks"]
    assert [g["rank"] for g in ranks] == list(range(n))
    assert all(set(g) == {"rank", "device", "pci", "uuid", "el_s", "avg_launch_us"} for g in ranks)
    assert len({g["pci"] for g in ranks}) == n


def test_distinct_device_check():
    """Two ranks on one PCI function fail the run unless --share-device."""
    sys.path.insert(0, ROOT)
    import bench
    same = [{"rank": 0, "pci": "0000:05:00", "uuid": "u"}, {"rank": 1, "pci": "0000:05:00", "uuid": "u"}]
    assert "share device" in bench.check_distinct_devices(same, False)
    assert bench.check_distinct_devices(same, True) is None
    other = [{"rank": 0, "pci": "0000:05:00", "uuid": "u"}, {"rank": 1, "pci": "0000:15:00", "uuid": "v"}]
    assert bench.check_distinct_devices(other, False) is None


def test_one_gpu_line_shape_unchanged():
    r = _bench("--gpus", "1", "--launch-dry-run", "--reads", "5000", "--no-cpu-baseline")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1
    assert set(line) - {"dry_run"} == LINE_KEYS
    assert "rccl_ranks" not in line["config"]   # only N > 1 lines carry it
    assert "ranks" not in line["config"]


def test_one_gpu_line_cpu_baseline_keys():
    """The one-GPU line's CPU leg (no device needed): the oracle on this GPU's
    CPU share, on one thread, and on every visible core (VERDICT r5 item 5:
    SURVEY §8d's threads = nproc), with the C1 and reference-architecture legs."""
    r = _bench("--gpus", "1", "--launch-dry-run", "--reads", "5000", "--cpu-seconds", "0.3",
               "--cpu-reads", "20000")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    cb = line["cpu_baseline"]
    assert {"value", "cores", "kind", "value_1thread", "value_allcores", "cores_allcores",
            "cpu_quota_cores", "c1_stats_mreads_s", "refarch", "sample"} <= set(cb)
    assert cb["cores_allcores"] == len(os.sched_getaffinity(0)) and cb["value_allcores"] > 0
    assert cb["kind"] == "port" and "visible cores" in cb["sample"]


def test_gpus_world_size_mismatch_fails():
    r = _bench("--gpus", "1", "--launch-dry-run", env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
    r = _bench("--gpus", "4", "--launch-dry-run", env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0


def test_failing_rank_fails_the_launch():
    # every rank refuses (--config dropin is a one-GPU harness): the launcher
    # reports the failure and prints no line
    r = _bench("--gpus", "2", "--config", "dropin")
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_one_failing_rank_ends_the_others():
    """Only rank 1 fails, before the rendezvous rank 0 is waiting in: the
    launcher sees it (it polls every rank, not up to the first running one),
    ends rank 0 and exits non-zero within seconds -- on a GPU box rank 0 would
    otherwise wait out the gloo timeout."""
    import time
    t0 = time.time()
    r = _bench("--gpus", "2", "--launch-dry-run", "--reads", "5000", "--dry-run-fail-rank", "1")
    assert r.returncode != 0
    assert "rank 1 fails" in r.stderr
    assert time.time() - t0 < 120
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpu_run_refuses_missing_devices():
    """A rank on a host without enough devices exits non-zero before any
    kernel (here: no device at all, without --share-device)."""
    r = _bench("--gpus", "1", "--no-cpu-baseline", "--no-e2e", "--reads", "1000", "--batch-reads", "1000")
    assert r.returncode != 0
