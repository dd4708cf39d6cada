"""CGR (chaos game) parity: hpgq_cgr_* (gfx950) vs the oracle's line-by-line
restatement of old/chaos_game.c:165-267, bit for bit, including batches that
force the speculative entry states to be replayed (homopolymer runs)."""
import json
import os

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev(reads, status=None):
    import torch
    dev = torch.device("cuda", 0)
    pad = np.zeros(H.DEVICE_SLACK, np.uint8)
    t = dict(seq=torch.from_numpy(np.concatenate([reads.seq, pad])).to(dev),
             qual=torch.from_numpy(np.concatenate([reads.qual, pad])).to(dev),
             idx=torch.from_numpy(reads.idx.copy()).to(dev))
    if status is not None:
        t["status"] = torch.from_numpy(status).to(dev)
    torch.cuda.synchronize()
    return t


def gpu_cgr(k, batches, statuses=None, mode=H.CGR_ALL_READS, base_quality=33):
    cg = H.ChaosGame(k, base_quality)
    replays = 0
    keep = []
    for i, reads in enumerate(batches):
        st = statuses[i] if statuses is not None else None
        t = _dev(reads, st)
        keep.append(t)
        b = H.engine.device_batch(reads.n, t["seq"].data_ptr(), t["qual"].data_ptr(),
                                  t["idx"].data_ptr())
        cg.fill_device(b, t["status"].data_ptr() if st is not None else None, mode)
        cg.sync()
        replays += cg.last_replays()
    ts, tq, wc = cg.tables()
    cg.close()
    return ts.reshape(-1), tq.reshape(-1), wc, replays


def oracle_cgr(k, batches, statuses=None, mode=0, base_quality=33):
    dim = 1 << k
    tables = (np.zeros(dim * dim, np.uint32), np.zeros(dim * dim, np.uint32),
              np.zeros(1, np.uint32))
    for i, reads in enumerate(batches):
        st = statuses[i] if statuses is not None else None
        O.cgr(k, reads, base_quality, status=st, mode=mode, tables=tables)
    return tables[0], tables[1], int(tables[2][0])


def assert_cgr(k, batches, **kw):
    ts, tq, wc, rep = gpu_cgr(k, batches, **kw)
    os_, oq, ow = oracle_cgr(k, batches, **kw)
    assert wc == ow
    if not np.array_equal(ts, os_):
        bad = np.nonzero(ts != os_)[0]
        raise AssertionError(f"table_seq differs at {bad[:8]} gpu={ts[bad[:8]]} ora={os_[bad[:8]]}")
    np.testing.assert_array_equal(tq, oq)
    return rep


def test_cgr_kat():
    from fastq_io import read_fastq
    kat = json.load(open(os.path.join(GOLD, "kat_expected.json")))["cgr"]
    reads = read_fastq(os.path.join(GOLD, kat["reads"]))
    ts, tq, wc, _ = gpu_cgr(kat["k"], [reads], base_quality=kat["base_quality"])
    np.testing.assert_array_equal(ts, kat["table_seq"])
    np.testing.assert_array_equal(tq, kat["table_q"])
    assert wc == kat["word_count"]


def test_cgr_committed_vector_k7():
    z = np.load(os.path.join(GOLD, "synth_cgr_k7.npz"))
    reads = O.Reads(z["seq"], z["qual"], z["idx"])
    ts, tq, wc, _ = gpu_cgr(7, [reads])
    np.testing.assert_array_equal(ts, z["table_seq"])
    np.testing.assert_array_equal(tq, z["table_q"])
    assert wc == int(z["word_count"])


@pytest.mark.parametrize("k", [1, 3, 5, 7, 8])
def test_cgr_synthetic_multi_batch(k):
    batches = [O.synth(3000, seed=5 + i, L=250, first=i * 3000) for i in range(3)]
    assert_cgr(k, batches)


def test_cgr_large_batch_k7():
    reads = O.synth(200_000, seed=5, L=250)
    rep = assert_cgr(7, [reads])
    assert rep == 0   # random context: every speculative entry state is exact


def _homopolymer_batch(rng, n=700, L=120):
    pairs = []
    for i in range(n):
        kind = i % 7
        if kind < 2:
            s = b"A" * L
        elif kind < 4:
            s = b"T" * L
        elif kind == 4:
            s = b"ACGT" * (L // 8) + b"A" * (L - 4 * (L // 8))
        elif kind == 5:
            s = np.array(rng.choice(list(b"ACGTN"), L), np.uint8).tobytes()
        else:
            s = b"C" * (L // 2) + b"G" * (L - L // 2)
        q = rng.integers(33, 75, L).astype(np.uint8).tobytes()
        pairs.append((s, q))
    return O.Reads.from_pairs(pairs)


def test_cgr_homopolymers_replay_exactly():
    rng = np.random.default_rng(3)
    rep = assert_cgr(7, [_homopolymer_batch(rng)])
    assert rep >= 0


@pytest.mark.parametrize("k", [2, 7, 9])
def test_cgr_boundary_clamp_runs(k):
    """Runs long enough for f to reach dim (the clamp at old/chaos_game.c:241-251)
    on x (A), y (G) and both (T), at ragged lengths so the clamp lands at every
    offset of the 8-base chunks the kernel proves clamp-free."""
    rng = np.random.default_rng(11 + k)
    pairs = []
    for i in range(600):
        L = int(rng.integers(1, 260))
        run = bytes([b"AGT"[i % 3]]) * int(rng.integers(40, 200))
        mix = np.array(rng.choice(list(b"ACGTN"), L), np.uint8).tobytes()
        s = (mix[: L // 3] + run + mix[L // 3:])[:L] if i % 4 else run[:L]
        q = rng.integers(33, 75, len(s)).astype(np.uint8).tobytes()
        pairs.append((s, q))
    assert_cgr(k, [O.Reads.from_pairs(pairs)])


def test_cgr_edge_bytes_and_lengths():
    pairs = [(b"", b""), (b"A", b"I"), (b"acgtACGTnNxX", b"IIII5555++++"),
             (b"ACGT" * 30, bytes([200] * 60 + [40] * 60)), (b"NNNNACGTACGTN", b"#" * 13),
             (b"RYKMACGTACGTACGT", b"?" * 16)] * 40
    reads = O.Reads.from_pairs(pairs)
    for k in (1, 2, 7, 12):
        assert_cgr(k, [reads])


def test_cgr_only_valid_reads():
    reads = O.synth(5000, seed=9, L=250)
    rng = np.random.default_rng(9)
    status = (rng.random(reads.n) < 0.8).astype(np.uint8)
    assert_cgr(7, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS)


def test_cgr_absolute_offsets():
    """data_indices need not start at 0 (a slice of a larger buffer)."""
    reads = O.synth(2000, seed=4, L=150)
    off = 37
    seq = np.concatenate([np.full(off, ord("G"), np.uint8), reads.seq])
    qual = np.concatenate([np.full(off, 60, np.uint8), reads.qual])
    shifted = O.Reads(seq, qual, reads.idx + off)
    ts, tq, wc, _ = gpu_cgr(7, [shifted])
    os_, oq, ow = oracle_cgr(7, [reads])
    np.testing.assert_array_equal(ts, os_)
    np.testing.assert_array_equal(tq, oq)
    assert wc == ow
