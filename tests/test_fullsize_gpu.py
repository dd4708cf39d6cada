"""Full-size parity: the BASELINE.json configurations at the per-GPU sizes bench.py times.

bench.py runs C2 (100 M x 150 bp reads, stats + --read-quality-range 20, --read-length-range 50,),
C3 (100 M pairs), C4 (62.5 M reads, edit + stats) and C5 (25 M x 250 bp, chaos game k = 7) on
resident synthetic batches.  These tests run the same workloads (same counter-based generator,
same 10 M / 12.5 M / 5 M-read device batches) through the C-ABI and compare, bit for bit, the
whole job's counters (C5: tables and word count) and every mask / trim with the oracle over the
same reads.  The generator is a function of the read index, so the oracle regenerates any read
range on the host by itself: 625 k-read parts on a thread pool (oracle_run is reentrant; ctypes
drops the GIL), counters summed mod 2^64, CGR tables mod 2^32 (old/chaos_game.c:253-258).  The
counters must also not depend on the batching: the same reads run again as half-size
sub-batches through absolute offsets.
"""
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

POOL = max(1, min(16, os.cpu_count() or 1))   # the GPU's CPU share on the test box
PART = 625_000


def _device_batches(seed, L, reads, batch, mates):
    """bench.make_batches at rank 0: per batch and mate (seq, qual, idx) device tensors."""
    dev = torch.device("cuda", 0)
    out = []
    for lo in range(0, reads, batch):
        n = min(batch, reads - lo)
        per_mate = []
        for m in range(mates):
            s = H.Synth(seed, L, 5, 5, 1, 33, m)
            idx = np.zeros(n + 1, np.int32)
            H.check(H.lib.hpgq_synth_indices_host(C.byref(s), lo, n, idx.ctypes.data), "idx")
            nb = int(idx[-1])
            sq = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
            ql = torch.empty(nb + 64, dtype=torch.uint8, device=dev)
            ix = torch.from_numpy(idx).to(dev)
            torch.cuda.synchronize()
            H.check(H.lib.hpgq_synth_device(C.byref(s), lo, n, sq.data_ptr(), ql.data_ptr(),
                                            ix.data_ptr(), None), "synth")
            per_mate.append((sq, ql, ix))
        out.append((lo, n, per_mate))
    torch.cuda.synchronize()
    return out


def _run_gpu(params, batches, split=False):
    """Counters of the whole job, plus masks / trims per batch (host arrays)."""
    dev = torch.device("cuda", 0)
    nsets = 2 if params.paired else 1
    masks, trims = [], []
    with H.Engine(params) as e:
        for lo, n, mm in batches:
            mask = torch.empty(n, dtype=torch.uint8, device=dev)
            trim = torch.empty(n * nsets, dtype=torch.int32, device=dev)
            cuts = [0, n // 2, n] if split else [0, n]
            for a, b in zip(cuts[:-1], cuts[1:]):   # absolute offsets: idx + a
                bs = [H.engine.device_batch(b - a, sq.data_ptr(), ql.data_ptr(), ix.data_ptr() + 4 * a)
                      for sq, ql, ix in mm]
                # (paired trims: mate 2 at num_reads + i of each call, so only whole-batch calls)
                e.run_device(bs[0], bs[1] if nsets == 2 else None, mask.data_ptr() + a,
                             trim.data_ptr() + 4 * a if params.edit_on and (nsets == 1 or not split) else None)
            e.sync()
            masks.append(mask.cpu().numpy())
            trims.append(trim.cpu().numpy().view(np.uint32) if params.edit_on else None)
        return e.counters(), masks, trims


def _oracle_range(params, seed, L, lo, n, pool):
    """The oracle over reads [lo, lo + n) in PART-read parts: (mask, trim, counters)."""
    nsets = 2 if params.paired else 1

    def part(a):
        m = min(PART, lo + n - a)
        r1 = O.synth(m, seed=seed, L=L, mate=0, first=a)
        r2 = O.synth(m, seed=seed, L=L, mate=1, first=a) if nsets == 2 else None
        return O.run(params, r1, r2, nthreads=1)

    res = list(pool.map(part, range(lo, lo + n, PART)))
    ctr = np.zeros(H.counters_len(params.lmax) * nsets, np.uint64)
    for _m, _t, c in res:
        ctr += c   # u64: wraps like the device counters
    # trims: [mate 1 | mate 2] per part -> [mate 1 of the range | mate 2 of the range]
    trim = np.concatenate([t[: len(t) // nsets * (mt + 1)][len(t) // nsets * mt:]
                           for mt in range(nsets) for _m, t, _c in res])
    return np.concatenate([m for m, _t, _c in res]), trim, ctr


def _check_config(params, seed, L, reads, batch):
    nsets = 2 if params.paired else 1
    batches = _device_batches(seed, L, reads, batch, nsets)
    c_gpu, masks, trims = _run_gpu(params, batches)
    want = np.zeros_like(c_gpu)
    with ThreadPoolExecutor(POOL) as pool:
        for (lo, n, _mm), m_g, t_g in zip(batches, masks, trims):
            m_o, t_o, c_o = _oracle_range(params, seed, L, lo, n, pool)
            np.testing.assert_array_equal(m_g, m_o, err_msg=f"mask of batch at {lo}")
            if params.edit_on:
                np.testing.assert_array_equal(t_g, t_o, err_msg=f"trim of batch at {lo}")
            want += c_o
    if not np.array_equal(c_gpu, want):
        bad = np.nonzero(c_gpu != want)[0]
        raise AssertionError(f"counters differ at {bad[:10]}: gpu {c_gpu[bad[:10]]} oracle {want[bad[:10]]}")
    assert int(c_gpu[H.S_NUM_INPUT]) == reads
    # the batching does not change the counters (half-size sub-batches, absolute offsets)
    c_split, _m, _t = _run_gpu(params, batches, split=True)
    np.testing.assert_array_equal(c_split, c_gpu)
    return c_gpu


def test_c2_full_size():
    """C2: 100 M x 150 bp in 10 M-read batches (bench --config c2)."""
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    c = _check_config(p, seed=2, L=150, reads=100_000_000, batch=10_000_000)
    assert 0 < int(c[H.S_NUM_FAILED]) < int(c[H.S_NUM_PASSED])


def test_c3_full_size():
    """C3: 100 M pairs, pair passes iff both mates pass (bench --config c3)."""
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    p.paired = 1
    _check_config(p, seed=3, L=150, reads=100_000_000, batch=10_000_000)


def test_c4_full_size():
    """C4: 62.5 M reads, edit (5'/3' Q20 trims) + stats in 12.5 M-read batches (bench --config c4)."""
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,")
    c = _check_config(p, seed=4, L=150, reads=62_500_000, batch=12_500_000)
    assert int(c[H.S_NUM_EDITED]) > 0


def test_c4_noor_full_size():
    """C4 flags + --max-N 2 (the post-trim N filter, src/edit_fastq.c:159-164) on the
    segmented edit kernel's N / out-of-range variant (bench --config c4_noor)."""
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", max_N=2)
    with H.Engine(p) as e:
        assert "edit" in e.kernel_name and "noor" in e.kernel_name, e.kernel_chain
    c = _check_config(p, seed=4, L=150, reads=62_500_000, batch=12_500_000)
    assert int(c[H.S_NUM_EDITED]) > 0 and int(c[H.S_NUM_FAILED]) > 0


def test_c4_pe_full_size():
    """C4 trims on paired-end 2 x 150: 50 M pairs in 10 M-pair batches, each mate
    trimmed, a pair kept iff both mates pass (bench --config c4_pe)."""
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", read_quality_range="20,")
    p.paired = 1
    with H.Engine(p) as e:
        assert "engine_tri_kernel" in e.kernel_name and "edit" in e.kernel_name, e.kernel_chain
    c = _check_config(p, seed=4, L=150, reads=50_000_000, batch=10_000_000)
    ln = H.counters_len(150)
    assert int(c[H.S_NUM_EDITED]) > 0 and int(c[ln + H.S_NUM_EDITED]) > 0


def test_c5_full_size():
    """C5: chaos game k = 7 over 25 M x 250 bp, one fill call per 5 M-read batch (bench
    --config c5): device tables == the oracle's chaos_game_fill_tables restatement summed
    over the same calls, every call on the stream pass (random reads: no exact replay)."""
    k, seed, L, reads, batch = 7, 5, 250, 25_000_000, 5_000_000
    batches = _device_batches(seed, L, reads, batch, 1)
    cg = H.ChaosGame(k, 33)
    try:
        for _lo, n, mm in batches:
            sq, ql, ix = mm[0]
            cg.fill_device(H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr()))
            cg.sync()
            assert cg.last_exact() == 0
        ts, tq, wc = cg.tables()
    finally:
        cg.close()
    del batches

    def call(lo):   # one fill call: fresh f state (old/chaos_game.c:180-181)
        r = O.synth(batch, seed=seed, L=L, first=lo)
        return O.cgr(k, r)

    with ThreadPoolExecutor(min(POOL, reads // batch)) as pool:
        res = list(pool.map(call, range(0, reads, batch)))
    want_s = np.zeros(1 << (2 * k), np.uint32)
    want_q = np.zeros(1 << (2 * k), np.uint32)
    want_w = 0
    for s, q, w in res:
        want_s += s
        want_q += q
        want_w = (want_w + int(w[0])) & 0xFFFFFFFF   # fq_word_count is u32
    np.testing.assert_array_equal(ts.reshape(-1), want_s)
    np.testing.assert_array_equal(tq.reshape(-1), want_q)
    assert wc == want_w


def test_c5_valid_full_size():
    """C5 in ONLY_VALID_READS mode with bench.py's 5 % invalid read_status
    (bench --config c5_valid): every call on the stream pass, tables equal the
    oracle's over the same calls and statuses (old/chaos_game.c:188)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import read_status
    k, seed, L, reads, batch = 7, 5, 250, 25_000_000, 5_000_000
    batches = _device_batches(seed, L, reads, batch, 1)
    cg = H.ChaosGame(k, 33)
    keep = []
    try:
        for lo, n, mm in batches:
            sq, ql, ix = mm[0]
            st = torch.from_numpy(read_status(n, seed, lo)).to(torch.device("cuda", 0))
            keep.append(st)
            cg.fill_device(H.engine.device_batch(n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr()),
                           st.data_ptr(), H.CGR_ONLY_VALID_READS)
            cg.sync()
            assert cg.last_exact() == 0
        ts, tq, wc = cg.tables()
    finally:
        cg.close()
    del batches, keep

    def call(lo):
        r = O.synth(batch, seed=seed, L=L, first=lo)
        return O.cgr(k, r, status=read_status(batch, seed, lo), mode=H.CGR_ONLY_VALID_READS)

    with ThreadPoolExecutor(min(POOL, reads // batch)) as pool:
        res = list(pool.map(call, range(0, reads, batch)))
    want_s = np.zeros(1 << (2 * k), np.uint32)
    want_q = np.zeros(1 << (2 * k), np.uint32)
    want_w = 0
    for s_, q, w in res:
        want_s += s_
        want_q += q
        want_w = (want_w + int(w[0])) & 0xFFFFFFFF
    np.testing.assert_array_equal(ts.reshape(-1), want_s)
    np.testing.assert_array_equal(tq.reshape(-1), want_q)
    assert wc == want_w
