"""Reads of any length: the stats merge, --kmers and the
CLI on reads of 1 .. 200,000 bases mixed with 150 bp reads, against the oracle.

The reference merges every position of every read into khash maps with no
length cap (src/stats_fastq.c:289-382) and grows each k-mer's counter_by_pos
with the read (:394-407).  libhpgq keeps lmax positions on chip and the rest in
its long-read tail: hpgq_read_counters gives the dense set (positions < lmax,
lengths <= lmax, every other entry of the long reads too, HPGQ_S_LONG_READS
counting them), which must equal the oracle at the ctx's lmax, and
hpgq_read_counters_ext the full set, which must equal the oracle at
lmax_ext = the longest merged read (where no read is long).  The device path
is run without a reservation (the tail's second pass inside hpgq_sync), with
hpgq_reserve_length, and through the host path (reserved from the batch's own
offsets); every route of the kernel chain meets the oracle.
"""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu

LONG = [1, 2, 5, 149, 150, 151, 157, 253, 1023, 1024, 1025, 1500, 4096, 70000, 200000]


def _read(rng, L, phred=33, kind=0):
    """One read: random bases (a few N, lowercase and IUPAC bytes), qualities
    good / bad / with low-quality ends, a few bytes >= 128 (signed char, Q13)."""
    s = rng.choice(np.frombuffer(b"ACGTACGTACGTACGTNacgR", np.uint8), L).astype(np.uint8)
    centre = 36 if kind % 3 else 12
    q = np.clip(centre + rng.integers(-6, 7, L), 2, 41) + phred
    if kind % 4 == 1 and L > 40:   # low-quality ends for the trims
        q[:min(L // 3, 30000)] = phred + 3
        q[-min(L // 4, 20000):] = phred + 4
    if kind % 7 == 2:
        q[rng.integers(0, L, max(1, L // 500))] = 200
    return bytes(s), bytes(q.astype(np.uint8))


def _mixed(seed, n150=3000, lens=LONG, phred=33):
    rng = np.random.default_rng(seed)
    pairs = [_read(rng, 150, phred, i) for i in range(n150)]
    for i, L in enumerate(lens):
        pairs.insert(int(rng.integers(0, len(pairs) + 1)), _read(rng, L, phred, i))
    return O.Reads.from_pairs(pairs)


def _ext_params(p, lmax_ext):
    q = H.Params.from_buffer_copy(p)
    q.lmax = lmax_ext
    return q


def _merged_max(params, reads, reads2, mask, trim):
    """The longest merged window (what lmax_ext must be)."""
    best = params.lmax
    if not params.stats_on:
        return best
    n = reads.n
    for m, r in enumerate([reads] + ([reads2] if reads2 is not None else [])):
        for i in range(n):
            if mask[i] != 1:
                continue
            t = int(trim[m * n + i]) if params.edit_on else 0
            w = int(r.idx[i + 1] - r.idx[i]) - (t & 0xFFFF) - (t >> 16)
            best = max(best, w)
    return best


def _check(params, reads, reads2, mask, trim, dense, ext, lmax_ext, info=""):
    m_o, t_o, c_o = O.run(params, reads, reads2)
    np.testing.assert_array_equal(mask, m_o, err_msg=info)
    if params.edit_on:
        np.testing.assert_array_equal(trim, t_o, err_msg=info)
    if not np.array_equal(dense, c_o):
        bad = np.nonzero(dense != c_o)[0]
        raise AssertionError(f"{info} dense counters differ at {bad[:10]}: {dense[bad[:10]]} vs {c_o[bad[:10]]}")
    want_L = _merged_max(params, reads, reads2, m_o, t_o)
    assert lmax_ext == want_L, (info, lmax_ext, want_L)
    _, _, c_x = O.run(_ext_params(params, lmax_ext), reads, reads2)
    assert int(c_x[H.S_LONG_READS]) == 0
    if not np.array_equal(ext, c_x):
        bad = np.nonzero(ext != c_x)[0]
        raise AssertionError(f"{info} full-length counters differ at {bad[:10]}: {ext[bad[:10]]} vs "
                             f"{c_x[bad[:10]]} (lmax_ext {lmax_ext})")


def _device(torch, reads):
    dev = torch.device("cuda", 0)
    sq = torch.from_numpy(np.concatenate([reads.seq, np.zeros(64, np.uint8)])).to(dev)
    ql = torch.from_numpy(np.concatenate([reads.qual, np.zeros(64, np.uint8)])).to(dev)
    ix = torch.from_numpy(reads.idx).to(dev)
    return (sq, ql, ix), H.engine.device_batch(reads.n, sq.data_ptr(), ql.data_ptr(), ix.data_ptr())


def _run(params, reads, reads2, path, route):
    """mask, trim, dense counters, (full-length counters, lmax_ext) through one path."""
    n, nm = reads.n, 2 if params.paired else 1
    with H.Engine(params, route=route) as e:
        if path == "host":
            b = H.engine.host_batch(reads.seq, reads.qual, reads.idx)
            b2 = H.engine.host_batch(reads2.seq, reads2.qual, reads2.idx) if reads2 is not None else None
            mask = np.zeros(n, np.uint8)
            trim = np.zeros(n * nm, np.uint32)
            e.run_host(b, b2, mask, trim)
            e.sync()
        else:
            torch = pytest.importorskip("torch")
            keep, b = _device(torch, reads)
            keep2, b2 = _device(torch, reads2) if reads2 is not None else (None, None)
            if path == "reserved":
                e.reserve_length(max(int(np.diff(r.idx).max()) for r in [reads] + ([reads2] if reads2 else [])))
            dm = torch.zeros(n, dtype=torch.uint8, device="cuda")
            dt = torch.zeros(n * nm, dtype=torch.int32, device="cuda")
            e.run_device(b, b2, dm.data_ptr(), dt.data_ptr())
            e.sync()   # (path "device": the tail's second pass runs here; the batch is still valid)
            mask = dm.cpu().numpy()
            trim = dt.cpu().numpy().view(np.uint32)
            del keep, keep2
        dense = e.counters()
        ext, L = e.counters_ext()
    return mask, trim, dense, ext, L


@pytest.mark.parametrize("route", ["auto", "single", "hex"])
@pytest.mark.parametrize("path", ["host", "device", "reserved"])
@pytest.mark.parametrize("lmax", [150, 1024])
def test_stats_any_length(route, path, lmax):
    reads = _mixed(1 + lmax)
    p = H.stats_params(lmax=lmax)
    _check(p, reads, None, *_run(p, reads, None, path, route), info=f"{route} {path} lmax {lmax}")


@pytest.mark.parametrize("path", ["host", "device"])
def test_stats_filter_any_length(path):
    reads = _mixed(7)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,", max_N=400)
    _check(p, reads, None, *_run(p, reads, None, path, "auto"), info=path)


@pytest.mark.parametrize("path", ["host", "device"])
def test_filter_only_any_length(path):
    reads = _mixed(8)
    p = H.filter_params(lmax=150, read_quality_range="20,", read_length_range="50,", max_N=400,
                        left_length=12, left_quality_range="20,")
    mask, _trim, dense, ext, L = _run(p, reads, None, path, "auto")
    m_o, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(mask, m_o)
    np.testing.assert_array_equal(dense, c_o)
    assert L == 150


@pytest.mark.parametrize("path", ["host", "device", "reserved"])
@pytest.mark.parametrize("paired", [0, 1])
def test_edit_stats_any_length(path, paired):
    reads = _mixed(11)
    reads2 = _mixed(12, lens=list(reversed(LONG))) if paired else None
    if paired:   # same read count, mate 2's own lengths
        assert reads2.n == reads.n
    p = H.edit_params(lmax=150, stats=True, left_length=40000, left_quality_range="20,",
                      right_length=30000, right_quality_range="20,", read_length_range="10,")
    p.paired = paired
    _check(p, reads, reads2, *_run(p, reads, reads2, path, "auto"), info=f"{path} paired {paired}")


def test_edit_trim_of_a_70000_base_low_quality_read():
    """a 70,000-base read whose every quality is low; both windows
    at their maximum (65,535): ts = 65,535, te = the 4,465 bases left, window
    empty -- and trims stay exact in 16 bits (HPGQ_MAX_EDIT_LENGTH)."""
    rng = np.random.default_rng(70)
    s = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 70000).astype(np.uint8))
    low = bytes([33 + 5]) * 70000
    half = bytes([33 + 5]) * 35000 + bytes([33 + 38]) * 35000   # a high-quality second half
    pairs = [(s, low), (s, half)] + O.synth(200, seed=70, L=150).pairs()
    reads = O.Reads.from_pairs(pairs)
    p = H.edit_params(lmax=1024, stats=True, left_length=65535, left_quality_range="20,",
                      right_length=65535, right_quality_range="20,")
    for path in ("host", "device"):
        mask, trim, dense, ext, L = _run(p, reads, None, path, "auto")
        assert int(trim[0]) & 0xFFFF == 65535 and int(trim[0]) >> 16 == 4465, hex(int(trim[0]))
        assert int(trim[1]) & 0xFFFF == 35000 and int(trim[1]) >> 16 == 0, hex(int(trim[1]))
        _check(p, reads, None, mask, trim, dense, ext, L, info=path)
        assert L == 35000   # read 2's window


def test_edit_length_over_65535_is_rejected():
    p = H.edit_params(lmax=150, left_length=100, left_quality_range="20,")
    p.edit_left_length = 65536
    with pytest.raises(H.HpgqError) as ei:
        H.Engine(p)
    assert ei.value.code == -1


def test_tail_second_pass_over_several_calls_and_reset():
    """Device calls without a reservation, some of them longer than the tail
    grown by an earlier second pass: each call's excess is merged once; a reset
    drops the pending second pass of the calls before it."""
    torch = pytest.importorskip("torch")
    parts = [_mixed(21, 500, [300, 2000]), _mixed(22, 500, [90000]), _mixed(23, 500, [5000, 120000])]
    p = H.stats_params(lmax=256, read_quality_range="5,")
    with H.Engine(p) as e:
        keep = []
        for r in parts[:2]:
            k, b = _device(torch, r)
            keep.append(k)
            e.run_device(b, None, None, None)
        e.reset()   # the first two calls are forgotten
        for r in parts:
            k, b = _device(torch, r)
            keep.append(k)
            e.run_device(b, None, None, None)
        dense = e.counters()
        ext, L = e.counters_ext()
    allr = O.Reads.from_pairs([pr for r in parts for pr in r.pairs()])
    m_o, t_o, c_o = O.run(p, allr)
    np.testing.assert_array_equal(dense, c_o)
    assert L == _merged_max(p, allr, None, m_o, t_o) == 90000   # (the 120,000-base read fails the filter)
    _, _, c_x = O.run(_ext_params(p, L), allr)
    np.testing.assert_array_equal(ext, c_x)


@pytest.mark.parametrize("reserve", [False, True])
@pytest.mark.parametrize("lmax", [3, 150, 1024])
def test_kmers_any_length(lmax, reserve):
    """--kmers: every start of every counted read (starts >= lmax - 4 in the
    tail); the full table equals the oracle's at npos_ext = longest - 4."""
    torch = pytest.importorskip("torch")
    reads = _mixed(31 + lmax)
    p = H.stats_params(lmax=lmax, read_quality_range="20,")
    m_o, _, _ = O.run(p, reads)
    mask = np.asarray(m_o, np.uint8)
    keep, b = _device(torch, reads)
    dm = torch.from_numpy(mask).cuda()
    km = H.Kmers(lmax)
    try:
        if reserve:
            km.reserve_length(int(np.diff(reads.idx).max()))
        km.count_device(b, dm.data_ptr())
        km.count_device(b, None)   # a second call, every read
        dense = km.by_pos()
        ext = km.by_pos_ext()
    finally:
        km.close()
    del keep
    want = O.kmers(reads, lmax, mask)
    O.kmers(reads, lmax, None, want)
    np.testing.assert_array_equal(dense, want)
    longest = int(np.diff(reads.idx).max())
    assert ext.shape == (1024, max(lmax, longest) - 4)
    want_x = O.kmers(reads, ext.shape[1] + 4, mask)
    O.kmers(reads, ext.shape[1] + 4, None, want_x)
    np.testing.assert_array_equal(ext, want_x)


def test_cli_long_reads(tmp_path):
    """The CLI on a FASTQ holding reads of 1 .. 90,000 bases: the counters dump
    (full length) equals the oracle's at the longest merged read, every report
    file equals the restatement of src/stats_report.c over it, and --kmers
    covers every start; filter and edit outputs are exact too."""
    from cli_lib import run_cli
    from fastq_io import to_fastq
    from oracle import report_ref
    reads = _mixed(41, 2000, [1, 2, 151, 1025, 1500, 4096, 90000])
    fq = tmp_path / "in.fq"
    fq.write_bytes(to_fastq(reads)[0])
    out = tmp_path / "out"
    out.mkdir()
    ctr, kb = tmp_path / "ctr.bin", tmp_path / "k.bin"
    run_cli(["stats", "-f", fq, "-o", out, "--read-quality-range", "20,", "--lmax", 150, "--chunk-mb", 1,
             "--counters-out", ctr, "--quiet"])
    p = H.stats_params(lmax=150, read_quality_range="20,")
    m_o, _, _ = O.run(p, reads)
    L = max([150] + [int(reads.idx[i + 1] - reads.idx[i]) for i in range(reads.n) if m_o[i]])
    got = np.fromfile(ctr, np.uint64)
    assert got.size == H.counters_len(L), (got.size, L)
    _, _, want = O.run(_ext_params(p, L), reads)
    np.testing.assert_array_equal(got, want)
    exp = report_ref.report_files(got, L, 33, "in.fq", {"filter_on": True, "read_quality_range": "20,"})
    for suffix, data in exp.items():
        assert (out / f"in.fq.{suffix}").read_bytes() == data, suffix
    kdir = tmp_path / "k"
    kdir.mkdir()
    run_cli(["stats", "-f", fq, "-o", kdir, "--read-quality-range", "20,", "--lmax", 150, "--chunk-mb", 1,
             "--kmers", "--kmers-out", kb, "--quiet"])
    kt = np.fromfile(kb, np.uint64).reshape(1024, -1)
    assert kt.shape[1] == L - 4
    np.testing.assert_array_equal(kt, O.kmers(reads, L, np.asarray(m_o, np.uint8)))
    # filter / edit: whole records, the long ones included
    run_cli(["filter", "-f", fq, "-o", tmp_path, "--read-quality-range", "20,", "--chunk-mb", 1, "--quiet"])
    pf = H.filter_params(lmax=1024, read_quality_range="20,")
    mf, _, _ = O.run(pf, reads)
    recs = []
    for i in range(reads.n):
        sq, ql = reads.read(i)
        recs.append(f"@r{i} extra:{i % 7}\n".encode() + sq + b"\n+\n" + ql + b"\n")
    assert (tmp_path / "passed.fq").read_bytes() == b"".join(r for r, m in zip(recs, mf) if m)
    assert (tmp_path / "failed.fq").read_bytes() == b"".join(r for r, m in zip(recs, mf) if not m)
    run_cli(["edit", "-f", fq, "-o", tmp_path, "--left-length", 40000, "--left-quality-range", "20,",
             "--right-length", 30000, "--right-quality-range", "20,", "--chunk-mb", 1, "--quiet"])
    pe = H.edit_params(lmax=1024, left_length=40000, left_quality_range="20,", right_length=30000,
                       right_quality_range="20,")
    me, te, _ = O.run(pe, reads)
    ok = []
    for i in range(reads.n):
        s, q = reads.read(i)
        ts, tend = int(te[i]) & 0xFFFF, int(te[i]) >> 16
        ok.append(f"@r{i} extra:{i % 7}\n".encode() + s[ts:len(s) - tend] + b"\n+\n" + q[ts:len(q) - tend] + b"\n")
    assert (tmp_path / "edit.fq").read_bytes() == b"".join(ok)
