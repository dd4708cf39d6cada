"""HIP engine parity: libhpgq (gfx950) vs the CPU oracle, bit for bit.

Every test runs the fused edit -> filter -> stats kernel through the C-ABI and
compares masks, trims and the packed u64 counters with oracle/liboracle.so on
the same seeded input (the oracle restates
src/stats_fastq.c:257-417 plus the build-defined filter/edit spec).
"""
import ctypes as C

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu


def gpu_host_path(params, reads, reads2=None):
    with H.Engine(params) as e:
        b2 = (reads2.seq, reads2.qual, reads2.idx) if reads2 is not None else (None,) * 3
        mask, trim = e.process(reads.seq, reads.qual, reads.idx, *b2)
        return mask, trim, e.counters()


def assert_same(params, reads, reads2=None, gpu=None):
    m_o, t_o, c_o = O.run(params, reads, reads2)
    m_g, t_g, c_g = gpu if gpu is not None else gpu_host_path(params, reads, reads2)
    np.testing.assert_array_equal(m_g, m_o)
    if params.edit_on:
        np.testing.assert_array_equal(t_g, t_o)
    if not np.array_equal(c_g, c_o):
        bad = np.nonzero(c_g != c_o)[0]
        raise AssertionError(f"counters differ at {bad[:10]} gpu={c_g[bad[:10]]} "
                             f"oracle={c_o[bad[:10]]} layout={H.layout(params.lmax)}")
    return c_o


STATS_CASES = {
    "stats": dict(),
    "c2_filter": dict(read_quality_range="20,", read_length_range="50,"),
    "all_filters": dict(read_length_range="60,140", read_quality_range="22,38", max_N=0,
                        max_out_of_quality=10, left_length=10, left_quality_range="25,",
                        right_length=15, right_quality_range="15,40"),
    "max_n": dict(max_N=1),
    "oor_only": dict(read_quality_range="10,35", max_out_of_quality=3),
}


@pytest.fixture(params=["auto", "tri", "wide", "single"])
def kernel_choice(request, monkeypatch):
    """Run a test with the default kernel chain (the segmented kernel in its
    16-byte-lane "hex" geometry first), with its 8-byte-lane "tri" or its
    4-segment "wide" geometry forced first and with the one-read-per-wave
    catch-all alone (hpgq_debug_set_route), so every kernel meets the oracle."""
    monkeypatch.setattr(H.engine, "DEFAULT_ROUTE", request.param)
    return request.param


@pytest.fixture(params=["auto", "tri", "wide"])
def geo_choice(request, monkeypatch):
    """The segmented kernel's geometries as the first stage (edit runs on all)."""
    monkeypatch.setattr(H.engine, "DEFAULT_ROUTE", request.param)
    return request.param


@pytest.mark.parametrize("name", sorted(STATS_CASES))
def test_stats_filter_synthetic(name, kernel_choice):
    reads = O.synth(20000, seed=2, L=150, trunc_pct=5, n_per_1024=8)
    p = H.stats_params(lmax=150, **STATS_CASES[name])
    c = assert_same(p, reads)
    assert c[H.S_NUM_INPUT] == reads.n


@pytest.mark.parametrize("L,lmax", [(160, 160), (157, 157), (156, 156), (150, 150), (60, 64), (3, 8)])
def test_tri_kernel_lengths(L, lmax, kernel_choice):
    reads = O.synth(7001, seed=12, L=L, trunc_pct=40, n_per_1024=30)
    p = H.stats_params(lmax=lmax, read_quality_range="18,", read_length_range="2,")
    assert_same(p, reads)


def test_filter_only_mask(kernel_choice):
    reads = O.synth(30000, seed=3, L=150, trunc_pct=10)
    p = H.filter_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    assert_same(p, reads)


@pytest.mark.parametrize("L,lmax", [(250, 250), (100, 256), (300, 512), (1000, 1024), (37, 40)])
def test_read_lengths(L, lmax):
    reads = O.synth(3000, seed=7, L=L, trunc_pct=30, n_per_1024=20)
    p = H.stats_params(lmax=lmax, read_quality_range="15,", read_length_range="30,")
    assert_same(p, reads)


def test_edit_trim_stats(geo_choice):
    reads = O.synth(20000, seed=4, L=150, trunc_pct=5)
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,")
    c = assert_same(p, reads)
    assert c[H.S_NUM_EDITED] > 0


@pytest.mark.parametrize("left,right", [(1, 1), (8, 31), (12, 32), (16, 32), (17, 33), (16, 0), (0, 32)])
def test_edit_window_sizes(left, right, geo_choice):
    """The trim at the window sizes where the kernel switches from one batch of
    loads (left <= 16, right <= 32) to the 8-byte loop, and (left <= 12) to the
    trims at the step, on reads as short as 0 -- the batch's first read 20
    bytes long, so its right window would begin before the buffer."""
    reads = O.synth(12000, seed=40 + left + right, L=150, trunc_pct=60)
    lowhi = bytes([33 + 5] * 7 + [33 + 30] * 6 + [33 + 8] * 7)
    reads = O.Reads.from_pairs([(b"ACGTN" * 4, lowhi)] + reads.pairs())
    kw = {}
    if left:
        kw.update(left_length=left, left_quality_range="22,")
    if right:
        kw.update(right_length=right, right_quality_range="18,36")
    p = H.edit_params(lmax=150, stats=True, **kw)
    c = assert_same(p, reads)
    assert c[H.S_NUM_EDITED] > 0


def test_edit_with_filter(geo_choice):
    reads = O.synth(20000, seed=5, L=150, trunc_pct=20)
    p = H.edit_params(lmax=150, stats=True, left_length=40, left_quality_range="30,",
                      right_length=60, right_quality_range="25,38",
                      read_length_range="60,", read_quality_range="20,", max_N=2)
    assert_same(p, reads)


def test_paired_end(geo_choice):
    r1 = O.synth(10000, seed=6, L=150, trunc_pct=5, mate=0)
    r2 = O.synth(10000, seed=6, L=150, trunc_pct=5, mate=1)
    assert np.array_equal(np.diff(r1.idx), np.diff(r2.idx))
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    p.paired = 1
    c = assert_same(p, r1, r2)
    ln = H.counters_len(150)
    assert c[H.S_NUM_PASSED] == c[ln + H.S_NUM_PASSED]


@pytest.mark.parametrize("left,right,lq,rq", [
    (1, 1, "22,", "18,36"), (8, 31, "22,35", "18,"), (13, 32, "22,", "18,36"), (16, 32, "20,30", "18,36"),
    (17, 33, "22,", "18,"), (16, 0, "22,35", None), (0, 32, None, "18,36"), (14, 20, "45,", "0,10")])
def test_paired_edit_window_sizes(left, right, lq, rq, geo_choice):
    """the paired-end trims -- the TDMA windows of the first stage
    (engine_tri_kernel<3, 2, edit, hex>), left lengths 13-16, bounded and empty
    ranges on both sides (the bounded-range branch), windows past the usual 16 /
    32 bytes, and each mate batch starting with a read shorter than 32 bytes
    (its right window would begin before the buffer)."""
    r1 = O.synth(6000, seed=50 + left + right, L=150, trunc_pct=60, mate=0)
    r2 = O.synth(6000, seed=50 + left + right, L=150, trunc_pct=60, mate=1)
    lowhi = bytes([33 + 5] * 7 + [33 + 30] * 6 + [33 + 8] * 7)
    r1 = O.Reads.from_pairs([(b"ACGTN" * 4, lowhi)] + r1.pairs())
    r2 = O.Reads.from_pairs([(b"TTGCA" * 3, lowhi[5:])] + r2.pairs())
    kw = {}
    if left:
        kw.update(left_length=left, left_quality_range=lq)
    if right:
        kw.update(right_length=right, right_quality_range=rq)
    p = H.edit_params(lmax=150, stats=True, **kw)
    p.paired = 1
    c = assert_same(p, r1, r2)
    assert c[H.S_NUM_EDITED] > 0
    if geo_choice == "auto":
        with H.Engine(p) as e:
            assert e.kernel_chain.startswith("hpgq::engine_tri_kernel<3, 2, edit, hex>"), e.kernel_chain


def test_paired_edit(geo_choice):
    r1 = O.synth(5000, seed=8, L=150, mate=0)
    r2 = O.synth(5000, seed=8, L=150, mate=1)
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", read_quality_range="25,")
    p.paired = 1
    assert_same(p, r1, r2)


def _edge_reads():
    rd = []
    rd.append((b"", b""))                                   # length 0
    rd.append((b"A", b"I"))                                 # length 1
    rd.append((b"GGGGCCCCGGGG", b"IIIIIIIIIIII"))           # GC 100
    rd.append((b"ATATATATAT", b"##########"))               # GC 0, Q2
    rd.append((b"NNNNNNNN", b"!!!!!!!!"))                   # all N, Q0
    rd.append((b"acgtnACGTN", b"IIIIIIIIII"))               # lowercase ignored
    rd.append((b"RYKMSWBDHV-.*ACGT", b"?" * 17))            # IUPAC / junk
    rd.append((b"ACGT" * 37 + b"AC", bytes(range(40, 190))))  # qualities >= 128
    rd.append((b"ACGTACGTAC", b"\xff\x80\x7f\x00\x01IIIII"))
    for L in (2, 3, 4, 5, 63, 64, 65, 127, 128, 129, 149, 150):
        rd.append(((b"CAGT" * 40)[:L], (b"5?I+" * 40)[:L]))
    return rd


@pytest.mark.parametrize("name", sorted(STATS_CASES))
def test_edge_reads(name, kernel_choice):
    reads = O.Reads.from_pairs(_edge_reads() * 7)
    p = H.stats_params(lmax=150, **STATS_CASES[name])
    assert_same(p, reads)


def test_edge_reads_edit_phred64(geo_choice):
    reads = O.Reads.from_pairs(_edge_reads() * 5)
    p = H.edit_params(lmax=150, stats=True, quality_encoding="phred64", left_length=5,
                      left_quality_range="0,10", right_length=7, right_quality_range="3,",
                      read_quality_range="1,")
    assert_same(p, reads)


def test_all_fail_and_empty_batch():
    reads = O.synth(5000, seed=9, L=150)
    p = H.stats_params(lmax=150, read_length_range="151,")
    c = assert_same(p, reads)
    assert c[H.S_NUM_PASSED] == 0
    empty = O.Reads(np.zeros(0, np.uint8), np.zeros(0, np.uint8), np.zeros(1, np.int32))
    with H.Engine(p) as e:
        mask, _ = e.process(empty.seq, empty.qual, empty.idx)
        assert e.counters().sum() == 0


def test_reads_longer_than_lmax_merge():
    """Reads longer than lmax are merged (round 6; the reference has no cap,
    src/stats_fastq.c:338-382): the dense set equals the oracle at lmax (the
    long reads' positions < lmax, bins and scalars, HPGQ_S_LONG_READS), the
    full-length set the oracle at the longest read (tests/test_longreads_gpu.py
    covers every path and length)."""
    reads = O.synth(100, seed=1, L=200)
    p = H.stats_params(lmax=150)
    with H.Engine(p) as e:
        e.process(reads.seq, reads.qual, reads.idx)
        dense = e.counters()
        ext, L = e.counters_ext()
    _, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(dense, c_o)
    assert int(dense[H.S_LONG_READS]) > 0 and L == 200
    p.lmax = 200
    _, _, c_x = O.run(p, reads)
    np.testing.assert_array_equal(ext, c_x)


def test_accumulates_across_batches_and_offsets(kernel_choice):
    """Counters merge over calls; data_indices need not start at 0."""
    reads = O.synth(12000, seed=10, L=150, trunc_pct=15)
    p = H.stats_params(lmax=150, read_quality_range="20,")
    _, _, c_o = O.run(p, reads)
    with H.Engine(p) as e:
        for lo, hi in [(0, 5000), (5000, 5001), (5001, 12000)]:
            idx = reads.idx[lo:hi + 1].copy()   # absolute offsets into the full buffers
            b = H.engine.host_batch(reads.seq, reads.qual, idx)
            mask = np.zeros(hi - lo, np.uint8)
            e.run_host(b, None, mask, None)
            e.sync()
        np.testing.assert_array_equal(e.counters(), c_o)


def test_device_path_torch_buffers(kernel_choice):
    torch = pytest.importorskip("torch")
    reads = O.synth(50000, seed=11, L=150, trunc_pct=5)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    dev = torch.device("cuda", 0)
    pad = np.zeros(H.DEVICE_SLACK, np.uint8)   # the C-ABI's readable slack
    seq = torch.from_numpy(np.concatenate([reads.seq, pad])).to(dev)
    qual = torch.from_numpy(np.concatenate([reads.qual, pad])).to(dev)
    idx = torch.from_numpy(reads.idx).to(dev)
    mask = torch.zeros(reads.n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    with H.Engine(p) as e:
        b = H.engine.device_batch(reads.n, seq.data_ptr(), qual.data_ptr(), idx.data_ptr())
        e.run_device(b, None, mask.data_ptr(), None)
        e.sync()
        gpu = (mask.cpu().numpy(), None, e.counters())
    assert_same(p, reads, gpu=gpu)


def test_synth_device_matches_oracle_generator():
    torch = pytest.importorskip("torch")
    n = 20000
    s = H.Synth(77, 150, 5, 5, 1, 33, 1)
    idx = np.zeros(n + 1, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), 1234, n, idx.ctypes.data), "idx")
    ref = O.synth(n, seed=77, L=150, trunc_pct=5, bad_pct=5, n_per_1024=1, mate=1, first=1234)
    np.testing.assert_array_equal(idx, ref.idx)
    dev = torch.device("cuda", 0)
    seq = torch.zeros(int(idx[-1]), dtype=torch.uint8, device=dev)
    qual = torch.zeros(int(idx[-1]), dtype=torch.uint8, device=dev)
    didx = torch.from_numpy(idx).to(dev)
    torch.cuda.synchronize()
    H.check(H.lib.hpgq_synth_device(C.byref(s), 1234, n, seq.data_ptr(), qual.data_ptr(),
                                    didx.data_ptr(), None), "synth")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(seq.cpu().numpy(), ref.seq)
    np.testing.assert_array_equal(qual.cpu().numpy(), ref.qual)


# ---- golden vectors: hand-derived KATs and the committed synthetic vectors ----
def _gold():
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("section", ["stats", "filter", "edit"])
def test_kat_gpu(section, kernel_choice):
    import json
    import os
    from fastq_io import read_fastq, check_partial
    kat = json.load(open(os.path.join(_gold(), "kat_expected.json")))
    reads = read_fastq(os.path.join(_gold(), kat["reads"]))
    lmax = kat["lmax"]
    if section == "stats":
        p = H.stats_params(lmax=lmax)
    elif section == "filter":
        p = H.stats_params(lmax=lmax, **kat["filter"]["flags"])
    else:
        p = H.edit_params(lmax=lmax, stats=True, **kat["edit"]["flags"])
    mask, trim, ctr = gpu_host_path(p, reads)
    exp = kat[section]
    check_partial(ctr, exp, lmax, H.layout(lmax))
    if "mask" in exp:
        np.testing.assert_array_equal(mask, exp["mask"])
    if "trim" in exp:
        np.testing.assert_array_equal(trim, exp["trim"])


@pytest.mark.parametrize("section", ["stats", "filter", "edit"])
def test_kat_signed_gpu(section, kernel_choice):
    """Quality bytes >= 128 count as signed `char` (src/stats_fastq.c:353-355,
    DESIGN.md Q13) on every kernel, by the hand-derived KAT."""
    import json
    import os
    from fastq_io import read_fastq, check_partial
    k = json.load(open(os.path.join(_gold(), "kat_expected.json")))["signed"]
    reads = read_fastq(os.path.join(_gold(), k["reads"]))
    lmax = k["lmax"]
    if section == "stats":
        p = H.stats_params(lmax=lmax)
    elif section == "filter":
        p = H.stats_params(lmax=lmax, **k["filter"]["flags"])
    else:
        p = H.edit_params(lmax=lmax, stats=True, **k["edit"]["flags"])
    mask, trim, ctr = gpu_host_path(p, reads)
    exp = k[section]
    check_partial(ctr, exp, lmax, H.layout(lmax))
    if "mask" in exp:
        np.testing.assert_array_equal(mask, exp["mask"])
    if "trim" in exp:
        np.testing.assert_array_equal(trim, exp["trim"])


@pytest.mark.parametrize("name", ["synth_c2_filter.npz", "synth_c4_edit.npz", "synth_c3_pe.npz",
                                  "synth_filter_all_250.npz"])
def test_committed_vectors_gpu(name, kernel_choice):
    import json
    import os
    z = np.load(os.path.join(_gold(), name))
    p = H.params_default(**json.loads(str(z["params"])))
    r1 = O.Reads(z["seq"], z["qual"], z["idx"])
    r2 = O.Reads(z["seq2"], z["qual2"], z["idx2"]) if p.paired else None
    mask, trim, ctr = gpu_host_path(p, r1, r2)
    np.testing.assert_array_equal(mask, z["mask"])
    np.testing.assert_array_equal(ctr, z["counters"])
    if p.edit_on:
        np.testing.assert_array_equal(trim, z["trim"])


def test_rccl_allreduce_single_rank():
    """hpgq_comm_init + hpgq_allreduce on a one-rank communicator: the RCCL
    path bench.py takes at N > 1 (fold, in-place u64 sum) leaves the counters
    equal to the oracle's."""
    reads = O.synth(30000, seed=31, L=150)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    with H.Engine(p) as e:
        e.comm_init(1, 0, H.engine.comm_unique_id())
        e.process(reads.seq, reads.qual, reads.idx)
        e.allreduce()
        e.sync()
        got = e.counters()
    _, _, want = O.run(p, reads)
    np.testing.assert_array_equal(got, want)


# ---- many blocks per wave: the persistent grid's block pipeline ------------
# (next block's prologue and offsets fetched ahead; the small cases above give
# each wave at most one block)
@pytest.mark.parametrize("case", ["c2", "c4", "c3"])
def test_many_blocks_per_wave(case, geo_choice):
    n = 1_200_000 if case != "c3" else 600_000   # > 4096 waves x 48 reads x 3
    if case == "c4":
        p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                          right_length=30, right_quality_range="20,")
    else:
        p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    if case == "c3":
        p.paired = 1
        r1 = O.synth(n, seed=21, L=150, trunc_pct=5, mate=0)
        r2 = O.synth(n, seed=21, L=150, trunc_pct=5, mate=1)
        assert_same(p, r1, r2)
    else:
        assert_same(p, O.synth(n, seed=20, L=150, trunc_pct=5, n_per_1024=2))


@pytest.mark.parametrize("name", ["max_n", "oor_only"])
def test_n_oor_filters_route_to_segmented_kernel(name, geo_choice):
    """max_N / max_out_of_quality run on the segmented kernel's filter variant
    (a second per-step scan of N | out-of-range), bit-identical to the oracle,
    at a size that gives every wave several blocks."""
    p = H.stats_params(lmax=150, **STATS_CASES[name])
    with H.Engine(p) as e:
        assert "engine_tri_x_kernel" in e.kernel_name
        assert ("hex" if geo_choice == "auto" else geo_choice) in e.kernel_name
    assert_same(p, O.synth(600_000, seed=23, L=150, trunc_pct=5, n_per_1024=12))


WINDOW_CASES = {
    "c2_left10": dict(read_quality_range="20,", read_length_range="50,", left_length=10,
                      left_quality_range="20,"),
    "right30": dict(right_length=30, right_quality_range="18,35"),
    "both_wide": dict(left_length=40, left_quality_range="25,", right_length=100,
                      right_quality_range=",30"),
    "longer_than_reads": dict(left_length=300, left_quality_range="20,", right_length=1,
                              right_quality_range="5,"),
    "left16_n": dict(left_length=16, left_quality_range="28,", max_N=2),   # no scan on hex
    "with_n_oor": dict(read_quality_range="10,38", max_N=1, max_out_of_quality=10, left_length=10,
                       left_quality_range="20,", right_length=7, right_quality_range="12,"),
}


@pytest.mark.parametrize("name", sorted(WINDOW_CASES))
def test_window_filters_route_to_segmented_kernel(name, geo_choice):
    """The 5'/3' window filters (src/filter_fastq.c:140-145 args 6-11) run on the
    segmented kernel's window-scan variant, bit-identical to the oracle, at a
    size that gives every wave several blocks."""
    p = H.stats_params(lmax=150, **WINDOW_CASES[name])
    with H.Engine(p) as e:
        assert "engine_tri_x_kernel" in e.kernel_name and "window" in e.kernel_name, e.kernel_chain
        assert ("noor" in e.kernel_name) == (name in ("with_n_oor", "left16_n"))
        assert ("hex" if geo_choice == "auto" else geo_choice) in e.kernel_name
    assert_same(p, O.synth(600_000, seed=24, L=150, trunc_pct=5, n_per_1024=12))


def test_window_filters_paired(geo_choice):
    p = H.stats_params(lmax=150, **WINDOW_CASES["c2_left10"])
    p.paired = 1
    r1 = O.synth(300_000, seed=25, L=150, trunc_pct=5, mate=0)
    r2 = O.synth(300_000, seed=25, L=150, trunc_pct=5, mate=1)
    with H.Engine(p) as e:
        assert "window" in e.kernel_name, e.kernel_chain
    assert_same(p, r1, r2)


# ---- edit with the extra filter scans / paired-end edit (segmented) ---------
C4_TRIMS = dict(left_length=10, left_quality_range="20,", right_length=30, right_quality_range="20,")
EDIT_X_CASES = {
    "c4_noor": dict(max_N=2),
    "maxn_oor": dict(read_quality_range="22,38", max_N=0, max_out_of_quality=5),
    "oor_len": dict(read_length_range="40,140", read_quality_range="15,", max_out_of_quality=12),
    "plain": dict(read_quality_range="25,"),
}


@pytest.mark.parametrize("paired", [0, 1])
@pytest.mark.parametrize("name", sorted(EDIT_X_CASES))
def test_edit_filters_route_to_segmented_kernel(name, paired, geo_choice):
    """edit with --max-N / --max-out-of-quality (the post-trim filter,
    src/edit_fastq.c:159-164) and paired-end edit (old/main_hpg_fastq_old.c:728)
    run on the segmented kernels -- no catch-all -- bit-identical to the
    oracle (masks, trims of both mates, both counter sets), at a size that
    gives every wave several blocks."""
    p = H.edit_params(lmax=150, stats=True, **C4_TRIMS, **EDIT_X_CASES[name])
    p.paired = paired
    with H.Engine(p) as e:
        nx = name != "plain"
        assert ("engine_tri_x_kernel" if nx else "engine_tri_kernel") in e.kernel_name, e.kernel_chain
        assert "edit" in e.kernel_name and ("noor" in e.kernel_name) == nx, e.kernel_chain
        assert f", {1 + paired}, " in e.kernel_name, e.kernel_chain
        assert ("hex" if geo_choice == "auto" else geo_choice) in e.kernel_name
    n = 300_000 if paired else 600_000
    r1 = O.synth(n, seed=26, L=150, trunc_pct=10, n_per_1024=12, mate=0)
    r2 = O.synth(n, seed=26, L=150, trunc_pct=10, n_per_1024=12, mate=1) if paired else None
    c = assert_same(p, r1, r2)
    assert c[H.S_NUM_EDITED] > 0 and c[H.S_NUM_FAILED] > 0


@pytest.mark.parametrize("paired", [0, 1])
@pytest.mark.parametrize("left", [1, 7, 12, 13])
def test_edit_trims_at_the_step(left, paired, geo_choice):
    """Single-end edit on hex with a left length <= 12 and a right one <= 32
    (C4's shape; paired-end the same trims on the TDMA kernel) applies the trims at the step (tri_body ST: the stream loads
    the untrimmed read, each step shifts its reads by al + ts <= 15 bytes
    through the wave's LDS buffer); 13 and the other geometries take the
    prologue trims.  Low left qualities make most steps shift; a bounded
    right range takes the five-VALU compare; exact against the oracle."""
    p = H.edit_params(lmax=150, stats=True, left_length=left, left_quality_range="30,",
                      right_length=32, right_quality_range="25,38",
                      **(dict(read_quality_range="24,") if paired else {}))
    p.paired = paired
    with H.Engine(p) as e:   # (paired-end keeps the prologue trims: tools/probes/pe_st.patch)
        assert (", st>" in e.kernel_name) == (left <= 12 and geo_choice == "auto" and not paired), e.kernel_chain
    n = 100_000 if paired else 200_000
    r1 = O.synth(n, seed=31, L=150, trunc_pct=15, n_per_1024=8, mate=0)
    r2 = O.synth(n, seed=31, L=150, trunc_pct=15, n_per_1024=8, mate=1) if paired else None
    c = assert_same(p, r1, r2)
    assert c[H.S_NUM_EDITED] > 0


@pytest.mark.parametrize("paired", [0, 1])
def test_edit_with_window_filters_abi(paired, geo_choice):
    """Through the C-ABI a caller may combine edit with the 5'/3' window
    filters (the CLI's edit disables them, src/edit_fastq.c:159-164): the
    windows apply to the trimmed read, on the segmented window-scan variant."""
    p = H.edit_params(lmax=150, stats=True, **C4_TRIMS, read_quality_range="18,")
    p.filter_on = 1
    p.left_length, p.min_left_quality, p.max_left_quality = 12, 24, H.MAX_VALUE
    p.right_length, p.min_right_quality, p.max_right_quality = 20, 10, 38
    p.paired = paired
    with H.Engine(p) as e:
        assert "edit" in e.kernel_name and "window" in e.kernel_name, e.kernel_chain
    r1 = O.synth(100_000, seed=27, L=150, trunc_pct=10, mate=0)
    r2 = O.synth(100_000, seed=27, L=150, trunc_pct=10, mate=1) if paired else None
    assert_same(p, r1, r2)


def test_paired_edit_mixed_lengths(geo_choice):
    """Paired-end edit across the chain: pairs with a mate past the first
    geometry go to the wide follow-up or the catch-all, trimmed there."""
    r1 = _mixed(2000, 9, [60, 150, 158, 240, 400], [20, 40, 20, 15, 5])
    r2 = _mixed(2000, 10, [60, 150, 158, 240, 400], [20, 40, 20, 15, 5])
    p = H.edit_params(lmax=512, stats=True, **C4_TRIMS, max_N=1)
    p.paired = 1
    assert_same(p, r1, r2)


# ---- routing by the reads' actual lengths ---------------------
C2 = dict(read_quality_range="20,", read_length_range="50,")


def _mixed(n, seed, lengths, weights):
    """Reads whose lengths are drawn from `lengths` (synthetic bases/qualities)."""
    rng = np.random.default_rng(seed)
    ls = rng.choice(lengths, size=n, p=np.asarray(weights, float) / sum(weights))
    pairs = []
    for i, L in enumerate(ls):
        r = O.synth(1, seed=seed * 7919 + i, L=int(L), trunc_pct=0, n_per_1024=8)
        pairs.append((bytes(r.seq), bytes(r.qual)))
    return O.Reads.from_pairs(pairs)


def test_lmax1024_150bp_runs_segmented(kernel_choice):
    """The drop-in default (CLI --lmax 1024, INTEGRATION's p->lmax = 1024) on
    150 bp reads runs the segmented hex kernel, bit-identical to the oracle."""
    p = H.stats_params(lmax=1024, **C2)
    if kernel_choice == "auto":
        with H.Engine(p) as e:
            assert "engine_tri_kernel" in e.kernel_name and "hex" in e.kernel_name, e.kernel_chain
            assert "wide, follow" in e.kernel_chain and "engine_kernel" in e.kernel_chain
    assert_same(p, O.synth(200_000, seed=31, L=150, trunc_pct=5, n_per_1024=4))


@pytest.mark.parametrize("lmax", [250, 1024])
def test_250bp_reads(lmax, kernel_choice):
    """250 bp reads: wide geometry first (lmax 250) or deferred by hex to the
    wide follow-up stage (lmax 1024); C2 flags, stats."""
    p = H.stats_params(lmax=lmax, **C2)
    if kernel_choice == "auto":
        with H.Engine(p) as e:
            assert ("wide" in e.kernel_name) == (lmax == 250), e.kernel_chain
    assert_same(p, O.synth(120_000, seed=32, L=250, trunc_pct=10, n_per_1024=4))


@pytest.mark.parametrize("case", ["stats", "c2", "nx", "window", "filter_only", "edit"])
def test_mixed_length_batches(case, kernel_choice):
    """Every stage of the chain in one batch: 20..156 (hex), 157..252 (wide),
    253..1024 (catch-all pipeline), > 1260 (catch-all chunk loop)."""
    reads = _mixed(3000, 5, [40, 100, 150, 156, 157, 160, 200, 252, 253, 300, 700, 1024, 1300, 3000],
                   [10, 20, 40, 5, 5, 5, 10, 5, 5, 5, 3, 2, 1, 1])
    if case == "stats":   # long reads fail the length filter: no error, all stats exact
        p = H.stats_params(lmax=1024, read_length_range=",1024")
    elif case == "c2":
        p = H.stats_params(lmax=1024, read_quality_range="20,", read_length_range="50,1024")
    elif case == "nx":
        p = H.stats_params(lmax=1024, read_length_range=",1024", max_N=1, max_out_of_quality=40)
    elif case == "window":
        p = H.stats_params(lmax=1024, read_length_range=",1024", left_length=12, left_quality_range="22,",
                           right_length=20, right_quality_range="15,")
    elif case == "filter_only":   # no stats: every length is filtered, no error
        p = H.filter_params(lmax=150, read_quality_range="20,", read_length_range="50,", max_N=3)
    else:   # edit without stats: trims of every length
        p = H.edit_params(lmax=150, stats=False, left_length=10, left_quality_range="20,",
                          right_length=30, right_quality_range="20,")
    assert_same(p, reads)


def test_mixed_lengths_edit_stats(geo_choice):
    reads = _mixed(2000, 6, [60, 150, 158, 240, 400], [20, 40, 20, 15, 5])
    p = H.edit_params(lmax=512, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,")
    assert_same(p, reads)


def test_mixed_lengths_paired(geo_choice):
    r1 = _mixed(2000, 7, [100, 150, 200, 400], [30, 40, 20, 10])
    # mate 2: same count, its own lengths (a pair defers when either mate is long)
    r2 = _mixed(2000, 8, [100, 150, 200, 400], [30, 40, 20, 10])
    p = H.stats_params(lmax=1024, read_quality_range="15,", read_length_range="30,")
    p.paired = 1
    assert_same(p, r1, r2)


def test_long_read_over_65535_bases():
    """A read longer than 16 bits (the round-1 kernel packed the length into 16
    bits and misread it): stats merge it at full length; filter only -> the
    chunk loop filters it like the oracle."""
    big = O.synth(1, seed=3, L=65636, trunc_pct=0)
    small = O.synth(300, seed=4, L=150)
    reads = O.Reads.from_pairs([(bytes(big.seq), bytes(big.qual))] + small.pairs())
    p = H.stats_params(lmax=1024)
    with H.Engine(p) as e:
        e.process(reads.seq, reads.qual, reads.idx)
        dense = e.counters()
        ext, L = e.counters_ext()
    np.testing.assert_array_equal(dense, O.run(p, reads)[2])
    assert L == 65636
    p.lmax = L
    np.testing.assert_array_equal(ext, O.run(p, reads)[2])
    p = H.filter_params(lmax=150, read_quality_range="20,", max_N=100)
    assert_same(p, reads)


def test_failing_long_read_is_no_error():
    """A read longer than lmax that FAILS the filter is not merged, so the call
    succeeds (only a merged long read is an error)."""
    reads = O.Reads.from_pairs([(b"A" * 400, b"#" * 400)] + O.synth(100, seed=5, L=150).pairs())
    p = H.stats_params(lmax=150, read_quality_range="20,")
    c = assert_same(p, reads)
    assert c[H.S_LONG_READS] == 0


def test_allreduce_out_of_place_twice():
    """hpgq_allreduce is out of place: calling it twice, or running another batch
    after it, never counts a rank's reads twice."""
    reads = O.synth(20000, seed=33, L=150)
    p = H.stats_params(lmax=150, **C2)
    _, _, want = O.run(p, reads)
    with H.Engine(p) as e:
        e.comm_init(1, 0, H.engine.comm_unique_id())
        e.process(reads.seq, reads.qual, reads.idx)
        e.allreduce()
        e.allreduce()
        e.sync()
        np.testing.assert_array_equal(e.counters(), want)
        e.process(reads.seq, reads.qual, reads.idx)
        e.allreduce()
        e.sync()
        np.testing.assert_array_equal(e.counters(), 2 * want)


def test_adaptive_first_stage_switches_and_stays_exact():
    """A ctx that may see long reads (lmax 1024) keeps a hex-first and a
    wide-first chain and picks per call from the deferral report of earlier
    calls: batches of 250 bp reads, then 150 bp reads, then mixed, accumulate
    into one counter set bit-identical to the oracle whatever chain ran."""
    p = H.stats_params(lmax=1024, **C2)
    batches = [O.synth(40_000, seed=40 + i, L=250, trunc_pct=5) for i in range(20)]
    batches += [O.synth(40_000, seed=60 + i, L=150, trunc_pct=5) for i in range(20)]
    batches += [_mixed(3000, 80 + i, [100, 150, 250, 600], [30, 30, 30, 10]) for i in range(4)]
    want = np.zeros(H.counters_len(1024), np.uint64)
    with H.Engine(p) as e:
        assert "adaptive" in e.kernel_chain, e.kernel_chain
        for r in batches:
            m_g, _ = e.process(r.seq, r.qual, r.idx)
            m_o, _, c_o = O.run(p, r)
            np.testing.assert_array_equal(m_g, m_o)
            want += c_o
        np.testing.assert_array_equal(e.counters(), want)


def test_debug_set_route_on_a_live_ctx():
    """hpgq_debug_set_route re-plans a ctx between batches: the counters keep
    accumulating, every route meets the oracle and the first stage's kernel
    name follows the route; the library itself reads no routing environment."""
    import os
    os.environ["HPGQ_KERNEL"] = "single"       # (rounds <= 3 read these; now ignored)
    os.environ["HPGQ_TRI_GEO"] = "tri"
    try:
        p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
        parts = [O.synth(6000, seed=300 + i, L=150, trunc_pct=10, first=9000 * i) for i in range(4)]
        names = []
        with H.Engine(p) as e:
            names.append(e.kernel_name)
            for r, route in zip(parts, ["auto", "single", "tri", "wide"]):
                e.set_route(route)
                names.append(e.kernel_name)
                m, _ = e.process(r.seq, r.qual, r.idx)
                np.testing.assert_array_equal(m, O.run(p, r)[0])
            got = e.counters()
        np.testing.assert_array_equal(got, sum(O.run(p, r)[2] for r in parts))
        assert "hex" in names[0] and "hex" in names[1]   # the environment changed nothing
        assert names[2].startswith("hpgq::engine_kernel<")
        assert ", tri" in names[3] and ", wide" in names[4]
        assert H.lib.hpgq_debug_set_route(None, 0) == -1   # HPGQ_E_INVALID
        with H.Engine(p) as e2:
            assert H.lib.hpgq_debug_set_route(e2._h, 99) == -1
            assert "hex" in e2.kernel_name
    finally:
        del os.environ["HPGQ_KERNEL"]
        del os.environ["HPGQ_TRI_GEO"]
