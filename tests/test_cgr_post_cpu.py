"""CGR post-processing (old/chaos_game.c:269-593) through the C-ABI on the host:
genomic-signature files, the difference table, its mean / standard deviation,
quality normalisation and the PGM images, against the pure-Python restatement
(oracle/pyref.py cgr_*).  Host code only: these run without a GPU."""
import os
import sys

import numpy as np
import pytest

import hpgfastq as H

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyref as R  # noqa: E402


def _tables(k, seed):
    rng = np.random.default_rng(seed)
    cells = 1 << (2 * k)
    ts = rng.integers(0, 400, cells).astype(np.uint32)
    ts[rng.random(cells) < 0.1] = 0   # empty cells
    tq = (ts.astype(np.uint64) * rng.integers(33 * k, 75 * k, cells)).astype(np.uint32)
    tg = rng.integers(0, 300, cells).astype(np.uint32)
    return ts, tq, tg, int(ts.sum()), int(tg.sum()) + 17


@pytest.mark.parametrize("k", [1, 3, 5, 7, 8])
def test_table_dif_and_stats(k):
    ts, _tq, tg, fw, rw = _tables(k, k)
    d, hi, lo = H.cgr_table_dif(k, ts, fw, tg, rw)
    rd, rhi, rlo = R.cgr_table_dif(k, ts.tolist(), fw, tg.tolist(), rw)
    assert d.tolist() == rd
    assert (hi, lo) == (rhi, rlo)
    m, s = H.cgr_dif_stats(k, d)
    assert (m, s) == R.cgr_dif_stats(rd)   # same summation order: bit-identical doubles


def test_table_dif_rejects_empty_counts():
    ts, _tq, tg, _fw, rw = _tables(3, 1)
    with pytest.raises(H.HpgqError):
        H.cgr_table_dif(3, ts, 0, tg, rw)   # LOG_FATAL in the reference (:331-333)


@pytest.mark.parametrize("k", [2, 7])
def test_normalize_quality(k):
    ts, tq, _tg, _fw, _rw = _tables(k, 10 + k)
    assert H.cgr_normalize_quality(k, ts, tq).tolist() == R.cgr_normalize_quality(k, ts.tolist(), tq.tolist())


@pytest.mark.parametrize("k,norm", [(1, 3.7), (4, 128.0 / 3.1), (7, 0.75), (8, 256.0 / 62)])
def test_pgm_bytes(tmp_path, k, norm):
    ts, _tq, _tg, _fw, _rw = _tables(k, 20 + k)
    ts[0] = 1_000_000   # (uchar) wrap of a large pixel
    f = tmp_path / "t.pgm"
    H.cgr_write_pgm(str(f), k, ts, norm)
    assert f.read_bytes() == R.cgr_pgm(k, ts.tolist(), norm)


@pytest.mark.parametrize("k", [3, 7])
def test_gs_file_round_trip(tmp_path, k):
    ts, _tq, _tg, fw, _rw = _tables(k, 30 + k)
    f = tmp_path / "ref.gs"
    H.cgr_write_gs(str(f), k, ts, fw)
    raw = f.read_bytes()
    assert len(raw) == R.GS_HEADER_BYTES + 4 * ts.size
    assert raw == R.cgr_gs_bytes(ts.tolist(), k, fw, name=str(f).encode())
    t2, w2 = H.cgr_load_gs(str(f), k)
    assert np.array_equal(t2, ts) and w2 == fw


def test_load_gs_missing_or_short(tmp_path):
    with pytest.raises(H.HpgqError):
        H.cgr_load_gs(str(tmp_path / "nope.gs"), 7)
    f = tmp_path / "short.gs"
    f.write_bytes(b"\0" * 100)
    with pytest.raises(H.HpgqError):
        H.cgr_load_gs(str(f), 7)


@pytest.mark.parametrize("with_gs", [False, True])
def test_write_images(tmp_path, with_gs):
    k = 5
    ts, tq, tg, fw, rw = _tables(k, 40)
    d = H.cgr_table_dif(k, ts, fw, tg, rw)[0] if with_gs else None
    H.cgr_write_images(str(tmp_path), "/some/dir/sample.fq", k, ts, tq, fw, d)
    base = tmp_path / "sample.fq_k=5"
    mem = 1 << (2 * k)
    fq_norm = 128.0 / (fw / mem)
    assert (tmp_path / "sample.fq_k=5_FG.pgm").read_bytes() == R.cgr_pgm(k, ts.tolist(), fq_norm)
    qn = R.cgr_normalize_quality(k, ts.tolist(), tq.tolist())
    assert (tmp_path / "sample.fq_k=5_QQ.pgm").read_bytes() == R.cgr_pgm(k, qn, 256.0 / 62)
    dif = tmp_path / "sample.fq_k=5_FG_dif.pgm"
    assert dif.exists() == with_gs
    if with_gs:
        absd = [min(abs(int(v)), 255) for v in d]
        assert dif.read_bytes() == R.cgr_pgm(k, absd, 1.0)
    assert str(base)   # (names: <dir>/<fq file>_k=<k>_{FG,QQ,FG_dif}.pgm, old/chaos_game.h:45-48)
