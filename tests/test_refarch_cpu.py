"""oracle/refarch.c (the reference's stats architecture restated for the
cpu_baseline "refarch" figure: worker threads per 10,000-read batch, one
consumer merging base by base through hash maps, src/stats_fastq.c:202-417)
computes the same counters as the dense-array oracle, so the two CPU figures
bench.py reports time the same work."""
import ctypes as C

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

_lib = O._lib
_lib.refarch_stats.restype = C.c_int
_lib.refarch_stats.argtypes = [C.POINTER(H.Params), C.POINTER(H.Batch), C.c_int, C.c_int, C.c_void_p]


def _refarch(p, reads, batch=10_000, workers=2):
    ctr = np.zeros(H.counters_len(p.lmax), np.uint64)
    b = reads.batch()
    assert _lib.refarch_stats(C.byref(p), C.byref(b), batch, workers, ctr.ctypes.data) == 0
    return ctr


@pytest.mark.parametrize("cfg", ["c1", "c2"])
@pytest.mark.parametrize("workers,batch", [(2, 10_000), (1, 997), (5, 4096)])
def test_refarch_equals_oracle(cfg, workers, batch):
    reads = O.synth(30_000, seed=7, L=150, trunc_pct=5, bad_pct=5, n_per_1024=4)
    p = H.stats_params(lmax=150) if cfg == "c1" else \
        H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    ref = _refarch(p, reads, batch, workers)
    _m, _t, orc = O.run(p, reads)
    lmax = p.lmax
    for k in (H.S_NUM_INPUT, H.S_NUM_PASSED, H.S_NUM_FAILED, H.S_NUM_STATS):
        assert ref[k] == orc[k], k
    a, b = H.NUM_SCALARS, H.counters_len(lmax)   # every histogram and per-position array
    assert np.array_equal(ref[a:b], orc[a:b])


def test_refarch_refuses_unsupported_options():
    reads = O.synth(100, seed=1)
    p = H.stats_params(lmax=150, read_quality_range="20,", max_N=2)
    ctr = np.zeros(H.counters_len(150), np.uint64)
    assert _lib.refarch_stats(C.byref(p), C.byref(reads.batch()), 10_000, 2, ctr.ctypes.data) == -1
