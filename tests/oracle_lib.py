"""ctypes view of oracle/liboracle.so (the CPU checker; tests only)."""
import ctypes as C
import os

import numpy as np

import hpgfastq as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = C.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
_lib.oracle_run.restype = C.c_int
_lib.oracle_run.argtypes = [C.POINTER(H.Params), C.POINTER(H.Batch), C.POINTER(H.Batch),
                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
_lib.oracle_synth.restype = None
_lib.oracle_synth.argtypes = [C.POINTER(H.Synth), C.c_int64, C.c_int64, C.c_void_p,
                              C.c_void_p, C.c_void_p]
_lib.oracle_synth_length.restype = C.c_int32
_lib.oracle_synth_length.argtypes = [C.POINTER(H.Synth), C.c_int64]
_lib.oracle_cgr_fill.restype = C.c_int
_lib.oracle_cgr_fill.argtypes = [C.c_int, C.c_int, C.POINTER(H.Batch), C.c_void_p, C.c_int,
                                 C.c_void_p, C.c_void_p, C.c_void_p]
_lib.oracle_max_threads.restype = C.c_int


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Reads:
    """Host SoA batch: seq/qual uint8 + int32 data_indices."""

    def __init__(self, seq, qual, idx):
        self.seq, self.qual, self.idx = seq, qual, idx

    @property
    def n(self):
        return len(self.idx) - 1

    def batch(self):
        return H.engine.host_batch(self.seq, self.qual, self.idx)

    def read(self, i):
        a, b = self.idx[i], self.idx[i + 1]
        return bytes(self.seq[a:b]), bytes(self.qual[a:b])

    def pairs(self):
        return [self.read(i) for i in range(self.n)]

    @staticmethod
    def from_pairs(pairs):
        lens = [len(s) for s, _ in pairs]
        idx = np.zeros(len(pairs) + 1, dtype=np.int32)
        idx[1:] = np.cumsum(lens)
        seq = np.frombuffer(b"".join(s for s, _ in pairs) + b"\0", dtype=np.uint8)[:-1].copy()
        qual = np.frombuffer(b"".join(q for _, q in pairs) + b"\0", dtype=np.uint8)[:-1].copy()
        return Reads(seq, qual, idx)


def synth(n, seed=1, L=150, trunc_pct=5, bad_pct=5, n_per_1024=1, phred=33, mate=0, first=0):
    s = H.Synth(seed, L, trunc_pct, bad_pct, n_per_1024, phred, mate)
    idx = np.zeros(n + 1, dtype=np.int32)
    total = sum(_lib.oracle_synth_length(C.byref(s), first + i) for i in range(n)) if n < 2000 \
        else None
    if total is None:
        # upper bound: every read at full length
        total = n * L
    seq = np.zeros(max(total, 1), dtype=np.uint8)
    qual = np.zeros(max(total, 1), dtype=np.uint8)
    _lib.oracle_synth(C.byref(s), first, n, _p(seq), _p(qual), _p(idx))
    end = int(idx[-1])
    return Reads(seq[:end].copy() if end else seq[:0].copy(),
                 qual[:end].copy() if end else qual[:0].copy(), idx)


def run(params, reads, reads2=None, nthreads=0):
    nsets = 2 if params.paired else 1
    n = reads.n
    mask = np.zeros(n, dtype=np.uint8)
    trim = np.zeros(n * nsets, dtype=np.uint32)
    ctr = np.zeros(H.counters_len(params.lmax) * nsets, dtype=np.uint64)
    b = reads.batch()
    b2 = reads2.batch() if reads2 is not None else None
    rc = _lib.oracle_run(C.byref(params), C.byref(b), C.byref(b2) if b2 else None,
                         _p(mask), _p(trim), _p(ctr), nthreads)
    assert rc == 0, rc
    return mask, trim, ctr


def cgr(k, reads, base_quality=33, status=None, mode=0, tables=None):
    dim = 1 << k
    if tables is None:
        tables = (np.zeros(dim * dim, dtype=np.uint32), np.zeros(dim * dim, dtype=np.uint32),
                  np.zeros(1, dtype=np.uint32))
    ts, tq, wc = tables
    b = reads.batch()
    rc = _lib.oracle_cgr_fill(k, base_quality, C.byref(b), _p(status), mode, _p(ts), _p(tq),
                              _p(wc))
    assert rc == 0, rc
    return ts, tq, wc


_lib.oracle_kmers.argtypes = [C.POINTER(H.Batch), C.c_void_p, C.c_int, C.c_void_p]
_lib.oracle_kmers.restype = C.c_int


def kmers(reads, lmax, mask=None, by_pos=None):
    """oracle --kmers counts: [1024, lmax-4] uint64 (added into by_pos if given)."""
    npos = max(lmax - 4, 0)
    if by_pos is None:
        by_pos = np.zeros((1024, npos), dtype=np.uint64)
    b = reads.batch()
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    rc = _lib.oracle_kmers(C.byref(b), _p(m), lmax, _p(by_pos))
    assert rc == 0, rc
    return by_pos
