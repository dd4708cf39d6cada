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


def gpu_cgr(k, batches, statuses=None, mode=H.CGR_ALL_READS, base_quality=33,
            path=H.CGR_PATH_AUTO, exact_log=None):
    cg = H.ChaosGame(k, base_quality, path=path)
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
        if exact_log is not None:
            exact_log.append(cg.last_exact())
    ts, tq, wc = cg.tables()
    cg.close()
    return ts.reshape(-1), tq.reshape(-1), wc, replays


def oracle_cgr(k, batches, statuses=None, mode=0, base_quality=33, path=None, exact_log=None):
    dim = 1 << k
    tables = (np.zeros(dim * dim, np.uint32), np.zeros(dim * dim, np.uint32),
              np.zeros(1, np.uint32))
    for i, reads in enumerate(batches):
        st = statuses[i] if statuses is not None else None
        O.cgr(k, reads, base_quality, status=st, mode=mode, tables=tables)
    return tables[0], tables[1], int(tables[2][0])


def stream_gate(k, reads, status=None, mode=H.CGR_ALL_READS):
    """Whether a streamed fill hands the call to the exact simulation
    (hpgq_cgr_stream.h): over the COUNTED reads (ONLY_VALID_READS: status 1,
    old/chaos_game.c:188) in order, a run of >= 48-k D moves on an axis (A/T on
    x, G/T on y; N and skipped reads move nothing, so runs pass through them),
    a byte other than A/C/G/T/N, or a quality byte >= 128.  The kernel's gate
    is exactly this predicate (the exact run scan runs wherever a run could
    reach the bound).  k > 7: always the exact kernels."""
    if k > 7:
        return True
    a, b = int(reads.idx[0]), int(reads.idx[-1])
    seq, qual = reads.seq[a:b], reads.qual[a:b]
    if mode == H.CGR_ONLY_VALID_READS:
        keep = np.repeat(np.asarray(status) == 1, np.diff(reads.idx))
        seq, qual = seq[keep], qual[keep]
    if (qual >= 128).any() or (~np.isin(seq, np.frombuffer(b"ACGTN", np.uint8))).any():
        return True
    mv = seq[np.isin(seq, np.frombuffer(b"ACGT", np.uint8))]
    for dset in (b"AT", b"GT"):
        d = np.concatenate([[0], np.isin(mv, np.frombuffer(dset, np.uint8)).astype(np.int8), [0]])
        e = np.diff(d)
        if len(mv) and (np.nonzero(e == -1)[0] - np.nonzero(e == 1)[0]).max(initial=0) >= 48 - k:
            return True
    return False


def assert_cgr(k, batches, **kw):
    ts, tq, wc, rep = gpu_cgr(k, batches, **kw)
    os_, oq, ow = oracle_cgr(k, batches, **kw)
    assert wc == ow
    if not np.array_equal(ts, os_):
        bad = np.nonzero(ts != os_)[0]
        raise AssertionError(f"table_seq differs at {bad[:8]} gpu={ts[bad[:8]]} ora={os_[bad[:8]]}")
    np.testing.assert_array_equal(tq, oq)
    return rep


@pytest.mark.parametrize("case", ["cgr", "cgr_k2"])
def test_cgr_kat(case):
    from fastq_io import read_fastq
    kat = json.load(open(os.path.join(GOLD, "kat_expected.json")))[case]
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


@pytest.mark.parametrize("path", [H.CGR_PATH_AUTO, H.CGR_PATH_EXACT])
@pytest.mark.parametrize("k", [1, 3, 5, 7, 8])
def test_cgr_synthetic_multi_batch(k, path):
    batches = [O.synth(3000, seed=5 + i, L=250, first=i * 3000) for i in range(3)]
    log = []
    assert_cgr(k, batches, path=path, exact_log=log)
    # random reads: the stream pass is proven exact for k <= 7
    assert log == [0 if (path == H.CGR_PATH_AUTO and k <= 7) else 1] * 3


@pytest.mark.parametrize("path", [H.CGR_PATH_AUTO, H.CGR_PATH_EXACT])
def test_cgr_large_batch_k7(path):
    reads = O.synth(200_000, seed=5, L=250)
    log = []
    rep = assert_cgr(7, [reads], path=path, exact_log=log)
    assert rep == 0   # random context: every speculative entry state is exact
    assert log == [0 if path == H.CGR_PATH_AUTO else 1]


@pytest.mark.parametrize("k", [4, 7])
def test_cgr_stream_many_spans_per_wave(k):
    """150 MB in one call: more 16 KB spans than the grid has waves, so every
    wave walks a tile stream across span boundaries (next span's context,
    cursor and first tile fetched while the last tile is counted).  Property
    check against the exact GPU kernels (validated against the oracle above)
    at a size the CPU oracle would take minutes on."""
    reads = O.synth(600_000, seed=11, L=250)
    log = []
    ts, tq, wc, _ = gpu_cgr(k, [reads], exact_log=log)
    assert log == [0]   # the stream pass ran
    es, eq, ew, rep = gpu_cgr(k, [reads], path=H.CGR_PATH_EXACT)
    assert rep == 0
    assert wc == ew and wc > 0
    np.testing.assert_array_equal(ts, es)
    np.testing.assert_array_equal(tq, eq)


def _run_batch(rng, k, run_len, n=900, split=False):
    """Random reads with D-move runs of run_len on x (A/T), y (G/T) or both
    (T), N sprinkled inside the runs (N does not move f), some runs split
    across two reads (f is carried across reads), at random offsets."""
    pairs = []
    alph = {0: b"AT", 1: b"GT", 2: b"T"}
    i = 0
    while len(pairs) < n:
        L = int(rng.integers(30, 300))
        mix = np.array(rng.choice(list(b"ACGT"), L), np.uint8).tobytes()
        if i % 5 == 0:
            ax = (i // 5) % 3
            run = bytes(rng.choice(list(alph[ax]), run_len).astype(np.uint8))
            if i % 2:
                pos = sorted(rng.choice(run_len, 3, replace=False))
                run = run[:pos[0]] + b"N" + run[pos[0]:pos[1]] + b"NN" + run[pos[1]:]
            # a Z on that axis on both sides so the run is exactly run_len long
            z = {0: b"C", 1: b"A", 2: b"C"}[ax]
            if split:
                cut = int(rng.integers(1, len(run)))
                a = mix[: L // 2] + z + run[:cut]
                b = run[cut:] + z + mix[L // 2:]
                pairs.append((a, bytes(rng.integers(33, 75, len(a)).astype(np.uint8))))
                pairs.append((b, bytes(rng.integers(33, 75, len(b)).astype(np.uint8))))
                i += 1
                continue
            off = int(rng.integers(0, L))
            sq = mix[:off] + z + run + z + mix[off:]
        else:
            sq = mix
        pairs.append((sq, bytes(rng.integers(33, 75, len(sq)).astype(np.uint8))))
        i += 1
    return O.Reads.from_pairs(pairs)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("k", [1, 2, 4, 7])
def test_cgr_stream_threshold_runs(k, split):
    """Runs of 47-k toward-dim moves stay on the stream path (and match the
    oracle); runs of 48-k set the gate and the exact simulation redoes the
    call (hpgq_cgr_stream.h: the cell is provably (int)f below 50-k)."""
    rng = np.random.default_rng(100 + k + 7 * split)
    below = _run_batch(rng, k, 47 - k, split=split)
    at = _run_batch(rng, k, 48 - k, split=split)
    log = []
    assert_cgr(k, [below], exact_log=log)
    assert log == [0]
    log = []
    assert_cgr(k, [at], exact_log=log)
    assert log == [1]


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
    log = []
    rep = assert_cgr(7, [_homopolymer_batch(rng)], exact_log=log)
    assert rep >= 0
    assert log == [1]   # poly-A/T: the stream pass sets the gate


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
        log = []
        assert_cgr(k, [reads], exact_log=log)
        assert log == [1]   # lowercase / IUPAC / qualities >= 128: exact path


@pytest.mark.parametrize("skipped", [0.0, 0.05, 0.2, 0.9, 1.0])
@pytest.mark.parametrize("k", [3, 7])
def test_cgr_only_valid_reads(k, skipped):
    """ONLY_VALID_READS (old/chaos_game.c:188) on the stream pass: random
    reads stay on it whatever the share of skipped reads; status values other
    than 1 (VALID_READ) all skip."""
    reads = O.synth(20000, seed=9, L=250)
    rng = np.random.default_rng(9)
    status = np.where(rng.random(reads.n) < skipped, rng.choice([0, 2, 255], reads.n), 1).astype(np.uint8)
    log = []
    assert_cgr(k, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS, exact_log=log)
    assert log == [0]


def test_cgr_only_valid_reads_exact_path():
    reads = O.synth(5000, seed=9, L=250)
    rng = np.random.default_rng(9)
    status = (rng.random(reads.n) < 0.8).astype(np.uint8)
    log = []
    assert_cgr(7, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS, path=H.CGR_PATH_EXACT,
               exact_log=log)
    assert log == [1]


def _skip_batch(rng, k, run_len, n=900):
    """Reads with D-move runs of run_len split by 1-3 SKIPPED reads (status 0)
    that hold Z moves, long D runs, lowercase / IUPAC bytes and qualities
    >= 128 -- none of which may count -- plus skipped reads elsewhere."""
    alph = {0: b"AT", 1: b"GT", 2: b"T"}
    pairs, status = [], []

    def junk():
        L = int(rng.integers(0, 200))
        s = bytearray(np.array(rng.choice(list(b"ACGTNacgtRYK"), L), np.uint8).tobytes())
        if L > 80 and rng.random() < 0.5:
            a = int(rng.integers(0, L - 70))
            s[a:a + 70] = bytes([b"AGT"[int(rng.integers(0, 3))]]) * 70
        q = rng.integers(33, 256, L).astype(np.uint8).tobytes()
        return bytes(s), q

    i = 0
    while len(pairs) < n:
        L = int(rng.integers(30, 300))
        mix = np.array(rng.choice(list(b"ACGT"), L), np.uint8).tobytes()
        if i % 4 == 0:
            ax = (i // 4) % 3
            run = bytes(rng.choice(list(alph[ax]), run_len).astype(np.uint8))
            z = {0: b"C", 1: b"A", 2: b"C"}[ax]
            cut = int(rng.integers(1, len(run)))
            a = mix[: L // 2] + z + run[:cut]
            b = run[cut:] + z + mix[L // 2:]
            pairs.append((a, rng.integers(33, 75, len(a)).astype(np.uint8).tobytes()))
            status.append(1)
            for _ in range(int(rng.integers(1, 4))):
                pairs.append(junk())
                status.append(int(rng.choice([0, 2])))
            pairs.append((b, rng.integers(33, 75, len(b)).astype(np.uint8).tobytes()))
            status.append(1)
        elif i % 7 == 3:
            pairs.append(junk())
            status.append(0)
        else:
            pairs.append((mix, rng.integers(33, 75, L).astype(np.uint8).tobytes()))
            status.append(1)
        i += 1
    return O.Reads.from_pairs(pairs), np.array(status, np.uint8)


@pytest.mark.parametrize("k", [1, 2, 4, 7])
def test_cgr_valid_threshold_runs_across_skipped_reads(k):
    """Runs of 47-k / 48-k D moves split by skipped reads: f passes through a
    skipped read unchanged (:188), so the halves form one run -- 47-k stays on
    the stream pass and 48-k sets the gate, whatever the skipped reads hold."""
    rng = np.random.default_rng(300 + k)
    for run_len, gate in ((47 - k, 0), (48 - k, 1)):
        reads, status = _skip_batch(rng, k, run_len)
        assert stream_gate(k, reads, status, H.CGR_ONLY_VALID_READS) == bool(gate)
        log = []
        assert_cgr(k, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS, exact_log=log)
        assert log == [gate]


@pytest.mark.parametrize("k", [4, 7])
def test_cgr_valid_stream_many_spans(k):
    """150 MB in one ONLY_VALID_READS call with 5 % skipped reads (and 2 %
    skipped runs of 1-40 reads, so skipped stretches cover whole tiles and
    spans): the stream pass equals the exact GPU kernels."""
    reads = O.synth(600_000, seed=12, L=250)
    rng = np.random.default_rng(12)
    status = (rng.random(reads.n) >= 0.05).astype(np.uint8)
    for s0 in rng.integers(0, reads.n - 40, reads.n // 2000):
        status[s0:s0 + int(rng.integers(1, 41))] = 0
    log = []
    ts, tq, wc, _ = gpu_cgr(k, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS, exact_log=log)
    assert log == [0]
    es, eq, ew, _ = gpu_cgr(k, [reads], statuses=[status], mode=H.CGR_ONLY_VALID_READS,
                            path=H.CGR_PATH_EXACT)
    assert wc == ew and wc > 0
    np.testing.assert_array_equal(ts, es)
    np.testing.assert_array_equal(tq, eq)


def test_cgr_valid_without_status_counts_nothing():
    reads = O.synth(1000, seed=3, L=150)
    cg = H.ChaosGame(7, 33)
    t = _dev(reads)
    cg.fill_device(H.engine.device_batch(reads.n, t["seq"].data_ptr(), t["qual"].data_ptr(),
                                         t["idx"].data_ptr()), None, H.CGR_ONLY_VALID_READS)
    ts, tq, wc = cg.tables()
    cg.close()
    assert wc == 0 and not ts.any() and not tq.any()


@pytest.mark.parametrize("off", [37, 16384 - 5, 3 * 16384 + 9])
def test_cgr_absolute_offsets(off):
    """data_indices need not start at 0 (a slice of a larger buffer)."""
    reads = O.synth(2000, seed=4, L=150)
    seq = np.concatenate([np.full(off, ord("G"), np.uint8), reads.seq])
    qual = np.concatenate([np.full(off, 60, np.uint8), reads.qual])
    shifted = O.Reads(seq, qual, reads.idx + off)
    ts, tq, wc, _ = gpu_cgr(7, [shifted])
    os_, oq, ow = oracle_cgr(7, [reads])
    np.testing.assert_array_equal(ts, os_)
    np.testing.assert_array_equal(tq, oq)
    assert wc == ow


@pytest.mark.parametrize("L", [1, 5, 16, 17, 63, 150])
def test_cgr_stream_short_and_ragged_reads(L):
    """Many reads per 16-byte lane / per tile (the start-bitmap cursor loops),
    N-only reads (long transparent stretches), ragged lengths, k = 3 and 7."""
    rng = np.random.default_rng(L)
    pairs = []
    for i in range(6000):
        n = int(rng.integers(0, L + 1))
        sq = (b"N" * n) if i % 97 == 0 else np.array(rng.choice(list(b"ACGTN"), n, p=[.24, .24, .24, .24, .04]), np.uint8).tobytes()
        pairs.append((sq, bytes(rng.integers(33, 75, n).astype(np.uint8))))
    reads = O.Reads.from_pairs(pairs)
    for k in (3, 7):
        log = []
        assert_cgr(k, [reads], exact_log=log)
        assert log == [0]


def test_cgr_stream_long_n_stretch():
    """A 40 KB stretch of N (several spans with no move at all) between
    A-runs: the runs on either side are counted as one (N does not move f)."""
    rng = np.random.default_rng(5)
    mix = lambda n: np.array(rng.choice(list(b"ACGT"), n), np.uint8).tobytes()  # noqa: E731
    pairs = [(mix(200), b"I" * 200) for _ in range(50)]
    pairs.append((mix(50) + b"C" + b"A" * 25, b"I" * 76))
    pairs += [(b"N" * 200, b"#" * 200) for _ in range(200)]
    pairs.append((b"A" * 25 + b"C" + mix(50), b"I" * 76))
    pairs += [(mix(200), b"I" * 200) for _ in range(50)]
    reads = O.Reads.from_pairs(pairs)
    log = []
    assert_cgr(7, [reads], exact_log=log)
    assert log == [1]   # 50 A's across the N stretch >= 41
    pairs[50] = (pairs[50][0][:-10] + b"C" * 10, b"I" * 76)   # now 15 + 25 = 40 < 41
    reads = O.Reads.from_pairs(pairs)
    log = []
    assert_cgr(7, [reads], exact_log=log)
    assert log == [0]


def test_cgr_allreduce_single_rank():
    """hpgq_cgr_comm_init + hpgq_cgr_allreduce on a one-rank communicator (the
    path bench.py takes at N > 1): the u32 sum leaves the tables equal to the
    oracle's, tables() returns the reduced copy until the next fill, and a
    second all-reduce does not double count."""
    rng = np.random.default_rng(77)
    batches = [O.synth(20000, seed=int(s), L=150, n_per_1024=8) for s in rng.integers(1, 1000, 2)]
    cg = H.ChaosGame(7, 33)
    cg.comm_init(1, 0, H.engine.comm_unique_id())
    keep = []
    for reads in batches:
        t = _dev(reads)
        keep.append(t)
        cg.fill_device(H.engine.device_batch(reads.n, t["seq"].data_ptr(), t["qual"].data_ptr(),
                                             t["idx"].data_ptr()))
    cg.allreduce()
    cg.allreduce()
    ts, tq, wc = cg.tables()
    cg.close()
    os_, oq, ow = oracle_cgr(7, batches)
    assert wc == ow
    np.testing.assert_array_equal(ts.reshape(-1), os_)
    np.testing.assert_array_equal(tq.reshape(-1), oq)
