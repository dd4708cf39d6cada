"""Engine / ChaosGame: Python handles over libhpgq contexts.

Host arrays are numpy; device buffers are passed as raw pointers (ints), so a
caller may own HBM through torch, hipMalloc or anything else.  Mirrors the
reference's worker-stage call shape: one call per batch, counters merged on
the device until read back (src/stats_fastq.c:202-253).
"""
import ctypes as C

import numpy as np

from ._abi import (lib, check, Params, Batch, Summary, counters_len, CGR_ALL_READS, ROUTES)

# Kernel route for new Engines (tests / A/B: a key of ROUTES, or None for the
# library's automatic chain).  Applied through hpgq_debug_set_route: the
# library itself reads no routing choice from the environment.
DEFAULT_ROUTE = None


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def host_batch(seq, qual, idx):
    """hpgq_batch_t over host numpy arrays (uint8, uint8, int32 of n+1)."""
    assert seq.dtype == np.uint8 and qual.dtype == np.uint8 and idx.dtype == np.int32
    assert seq.flags.c_contiguous and qual.flags.c_contiguous and idx.flags.c_contiguous
    b = Batch(len(idx) - 1, seq.ctypes.data, qual.ctypes.data, idx.ctypes.data)
    b._keep = (seq, qual, idx)   # the struct holds raw pointers: keep the arrays alive with it
    return b


def device_batch(num_reads, seq_ptr, qual_ptr, idx_ptr):
    return Batch(int(num_reads), int(seq_ptr), int(qual_ptr), int(idx_ptr))


class Engine:
    """One hpgq_ctx: a HIP stream + device counters on `device`."""

    def __init__(self, params, device=0, route=None):
        if not isinstance(params, Params):
            raise TypeError("params must be hpgfastq.Params")
        self.params = params
        self.lmax = params.lmax
        self.nsets = 2 if params.paired else 1
        h = C.c_void_p()
        check(lib.hpgq_open(C.byref(h), device, C.byref(params)), "hpgq_open")
        self._h = h
        route = route if route is not None else DEFAULT_ROUTE
        if route is not None and route != "auto":
            self.set_route(route)

    def set_route(self, route):
        """hpgq_debug_set_route: 'auto', 'single' (catch-all alone), 'tri' /
        'hex' / 'wide' first, 'auto_fixed' (no adaptive first stage)."""
        check(lib.hpgq_debug_set_route(self._h, ROUTES[route]), "hpgq_debug_set_route")

    def close(self):
        if self._h:
            lib.hpgq_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib.hpgq_stream(self._h)

    @property
    def kernel_name(self):
        """The engine kernel instance this ctx launches."""
        return lib.hpgq_kernel_name(self._h).decode()

    @property
    def kernel_chain(self):
        """The ctx's kernel chain: first stage -> follow-up stages."""
        return lib.hpgq_kernel_chain(self._h).decode()

    def run_host(self, batch, batch2=None, mask=None, trim=None):
        """Host numpy batch; mask/trim are numpy outputs valid after sync()."""
        check(lib.hpgq_run_host(self._h, C.byref(batch), C.byref(batch2) if batch2 else None,
                                _ptr(mask), _ptr(trim)), "hpgq_run_host")

    def run_host_in_place(self, mates, mask=None, trim=None):
        """hpgq_host_batch + hpgq_run_host: each (seq u8, qual u8, idx i32 from 0)
        of `mates` is written straight into the ctx's staging slot (no copy in
        the library); mask/trim are numpy outputs valid after sync()."""
        bs = [Batch() for _ in mates]
        nb = [int(ix[-1]) for (_s, _q, ix) in mates]
        n = len(mates[0][2]) - 1
        check(lib.hpgq_host_batch(self._h, n, nb[0], nb[1] if len(mates) > 1 else 0, C.byref(bs[0]),
                                  C.byref(bs[1]) if len(mates) > 1 else None), "hpgq_host_batch")
        for b, (sq, ql, ix) in zip(bs, mates):
            C.memmove(b.data_indices, ix.ctypes.data, ix.nbytes)
            C.memmove(b.seq, sq.ctypes.data, int(ix[-1]))
            C.memmove(b.quality, ql.ctypes.data, int(ix[-1]))
        check(lib.hpgq_run_host(self._h, C.byref(bs[0]), C.byref(bs[1]) if len(mates) > 1 else None,
                                _ptr(mask), _ptr(trim)), "hpgq_run_host")

    def run_device(self, batch, batch2=None, mask_ptr=None, trim_ptr=None):
        check(lib.hpgq_run_device(self._h, C.byref(batch), C.byref(batch2) if batch2 else None,
                                  mask_ptr, trim_ptr), "hpgq_run_device")

    def sync(self):
        check(lib.hpgq_sync(self._h), "hpgq_sync")

    def reset(self):
        check(lib.hpgq_reset(self._h), "hpgq_reset")

    def reserve_length(self, max_len):
        """hpgq_reserve_length: the long-read tail for merged reads up to max_len."""
        check(lib.hpgq_reserve_length(self._h, int(max_len)), "hpgq_reserve_length")

    def counters(self):
        n = lib.hpgq_counters_size(self._h)
        out = np.zeros(n, dtype=np.uint64)
        check(lib.hpgq_read_counters(self._h, _ptr(out), n), "hpgq_read_counters")
        return out

    def counters_ext(self):
        """hpgq_read_counters_ext -> (counters of every merged read at full
        length in the layout of lmax_ext, lmax_ext).  Collective after
        allreduce() (every rank calls it)."""
        L = C.c_int32(0)
        check(lib.hpgq_read_counters_ext(self._h, None, 0, C.byref(L)), "hpgq_read_counters_ext")
        out = np.zeros(counters_len(L.value) * self.nsets, dtype=np.uint64)
        L2 = C.c_int32(0)
        check(lib.hpgq_read_counters_ext(self._h, _ptr(out), out.size, C.byref(L2)), "hpgq_read_counters_ext")
        assert L2.value == L.value
        return out, L.value

    def counters_device_ptr(self):
        return lib.hpgq_counters_device(self._h)

    def comm_init(self, nranks, rank, uid):
        check(lib.hpgq_comm_init(self._h, nranks, rank, uid), "hpgq_comm_init")

    def allreduce(self):
        check(lib.hpgq_allreduce(self._h), "hpgq_allreduce")

    def comm_count(self):
        """Ranks in the ctx's RCCL communicator (ncclCommCount)."""
        n = C.c_int(0)
        check(lib.hpgq_comm_count(self._h, C.byref(n)), "hpgq_comm_count")
        return n.value

    def process(self, seq, qual, idx, seq2=None, qual2=None, idx2=None):
        """Convenience: one host batch -> (mask, trim); counters accumulate."""
        n = len(idx) - 1
        b = host_batch(seq, qual, idx)
        b2 = host_batch(seq2, qual2, idx2) if self.params.paired else None
        mask = np.zeros(n, dtype=np.uint8)
        trim = np.zeros(n * self.nsets, dtype=np.uint32)
        self.run_host(b, b2, mask, trim)
        self.sync()
        return mask, trim


def comm_unique_id():
    buf = C.create_string_buffer(128)
    check(lib.hpgq_comm_unique_id(buf), "hpgq_comm_unique_id")
    return buf.raw


def summary(counter_set, lmax):
    s = Summary()
    arr = np.ascontiguousarray(counter_set[:counters_len(lmax)], dtype=np.uint64)
    check(lib.hpgq_counters_summary(_ptr(arr), lmax, C.byref(s)), "hpgq_counters_summary")
    return {f: getattr(s, f) for f, _ in Summary._fields_}


class ChaosGame:
    """hpgq_cgr: chaos_game_fill_tables on the device (old/chaos_game.c:165)."""

    def __init__(self, k, base_quality=33, device=0, path=0):
        self.k = k
        self.dim = 1 << k
        h = C.c_void_p()
        check(lib.hpgq_cgr_open(C.byref(h), device, k, base_quality), "hpgq_cgr_open")
        self._h = h
        check(lib.hpgq_cgr_set_path(h, path), "hpgq_cgr_set_path")

    def close(self):
        if self._h:
            lib.hpgq_cgr_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib.hpgq_cgr_stream(self._h)

    def fill_device(self, batch, status_ptr=None, mode=CGR_ALL_READS):
        check(lib.hpgq_cgr_fill_device(self._h, C.byref(batch), status_ptr, mode),
              "hpgq_cgr_fill_device")

    def sync(self):
        check(lib.hpgq_cgr_sync(self._h), "hpgq_cgr_sync")

    def reset(self):
        check(lib.hpgq_cgr_reset(self._h), "hpgq_cgr_reset")

    def comm_init(self, nranks, rank, uid):
        """RCCL communicator for the table sum (uid from comm_unique_id())."""
        check(lib.hpgq_cgr_comm_init(self._h, nranks, rank, uid), "hpgq_cgr_comm_init")

    def allreduce(self):
        """u32 sum of every rank's tables and word count (hpgq_cgr_allreduce);
        tables() returns it until the next fill or reset."""
        check(lib.hpgq_cgr_allreduce(self._h), "hpgq_cgr_allreduce")

    def comm_count(self):
        n = C.c_int(0)
        check(lib.hpgq_cgr_comm_count(self._h, C.byref(n)), "hpgq_cgr_comm_count")
        return n.value

    def last_replays(self):
        return int(lib.hpgq_cgr_last_replays(self._h))

    def last_exact(self):
        """1 if the last synced fill ran the exact double simulation, 0 if the
        stream pass was proven exact (hpgq_cgr_last_exact)."""
        return int(lib.hpgq_cgr_last_exact(self._h))

    def tables(self):
        cells = self.dim * self.dim
        ts = np.zeros(cells, dtype=np.uint32)
        tq = np.zeros(cells, dtype=np.uint32)
        wc = np.zeros(1, dtype=np.uint32)
        check(lib.hpgq_cgr_read(self._h, _ptr(ts), _ptr(tq), _ptr(wc)), "hpgq_cgr_read")
        return ts.reshape(self.dim, self.dim), tq.reshape(self.dim, self.dim), int(wc[0])


def cgr_write_gs(path, k, table, word_count):
    """hpgq_cgr_write_gs: a genomic-signature file (header_gs_t + dim*dim u32)."""
    t = np.ascontiguousarray(table, dtype=np.uint32).reshape(-1)
    check(lib.hpgq_cgr_write_gs(path.encode(), k, _ptr(t), word_count), "hpgq_cgr_write_gs")


def cgr_load_gs(path, k):
    """hpgq_cgr_load_gs -> (table u32 [dim*dim], ref_word_count)."""
    t = np.zeros(1 << (2 * k), dtype=np.uint32)
    w = np.zeros(1, dtype=np.uint32)
    check(lib.hpgq_cgr_load_gs(path.encode(), k, _ptr(t), _ptr(w)), "hpgq_cgr_load_gs")
    return t, int(w[0])


def cgr_table_dif(k, table_seq, fq_words, table_gs, ref_words):
    """hpgq_cgr_table_dif -> (int32 table_dif, highest, lowest)."""
    ts = np.ascontiguousarray(table_seq, dtype=np.uint32).reshape(-1)
    tg = np.ascontiguousarray(table_gs, dtype=np.uint32).reshape(-1)
    d = np.zeros(ts.size, dtype=np.int32)
    hl = np.zeros(2, dtype=np.int32)
    check(lib.hpgq_cgr_table_dif(k, _ptr(ts), fq_words, _ptr(tg), ref_words, _ptr(d),
                                 _ptr(hl), hl.ctypes.data + 4), "hpgq_cgr_table_dif")
    return d, int(hl[0]), int(hl[1])


def cgr_dif_stats(k, table_dif):
    d = np.ascontiguousarray(table_dif, dtype=np.int32).reshape(-1)
    ms = np.zeros(2, dtype=np.float64)
    check(lib.hpgq_cgr_dif_stats(k, _ptr(d), _ptr(ms), ms.ctypes.data + 8), "hpgq_cgr_dif_stats")
    return float(ms[0]), float(ms[1])


def cgr_normalize_quality(k, table_seq, table_q):
    ts = np.ascontiguousarray(table_seq, dtype=np.uint32).reshape(-1)
    tq = np.array(table_q, dtype=np.uint32).reshape(-1)
    check(lib.hpgq_cgr_normalize_quality(k, _ptr(ts), _ptr(tq)), "hpgq_cgr_normalize_quality")
    return tq


def cgr_write_pgm(path, k, table, norm):
    t = np.ascontiguousarray(table, dtype=np.uint32).reshape(-1)
    check(lib.hpgq_cgr_write_pgm(path.encode(), k, _ptr(t), norm), "hpgq_cgr_write_pgm")


def cgr_write_images(report_dir, fq_path, k, table_seq, table_q, fq_words, table_dif=None):
    """hpgq_cgr_write_images: <dir>/<fq>_k=<k>_FG.pgm, _QQ.pgm (+ _FG_dif.pgm)."""
    ts = np.ascontiguousarray(table_seq, dtype=np.uint32).reshape(-1)
    tq = np.array(table_q, dtype=np.uint32).reshape(-1)
    d = None if table_dif is None else np.ascontiguousarray(table_dif, dtype=np.int32).reshape(-1)
    check(lib.hpgq_cgr_write_images(report_dir.encode(), fq_path.encode(), k, _ptr(ts), _ptr(tq),
                                    fq_words, _ptr(d) if d is not None else None),
          "hpgq_cgr_write_images")


class Kmers:
    """hpgq_kmers: `stats --kmers` 5-mer counts per start position
    (merge src/stats_fastq.c:384-410; build-defined per-read rule)."""

    def __init__(self, lmax, device=0, stream=None):
        self.lmax = lmax
        self.npos = max(lmax - 4, 0)
        h = C.c_void_p()
        check(lib.hpgq_kmers_open(C.byref(h), device, lmax, stream), "hpgq_kmers_open")
        self._h = h

    def close(self):
        if self._h:
            lib.hpgq_kmers_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def count_device(self, batch, mask_ptr=None):
        check(lib.hpgq_kmers_count_device(self._h, C.byref(batch), mask_ptr),
              "hpgq_kmers_count_device")

    def sync(self):
        check(lib.hpgq_kmers_sync(self._h), "hpgq_kmers_sync")

    def reset(self):
        check(lib.hpgq_kmers_reset(self._h), "hpgq_kmers_reset")

    def by_pos(self):
        out = np.zeros((1024, self.npos), dtype=np.uint64)
        check(lib.hpgq_kmers_read(self._h, _ptr(out), out.size), "hpgq_kmers_read")
        return out

    def reserve_length(self, max_len):
        check(lib.hpgq_kmers_reserve_length(self._h, int(max_len)), "hpgq_kmers_reserve_length")

    def by_pos_ext(self):
        """hpgq_kmers_read_ext: every start, [1024, npos_ext]."""
        P = C.c_int32(0)
        check(lib.hpgq_kmers_read_ext(self._h, None, 0, C.byref(P)), "hpgq_kmers_read_ext")
        out = np.zeros((1024, P.value), dtype=np.uint64)
        check(lib.hpgq_kmers_read_ext(self._h, _ptr(out), out.size, C.byref(P)), "hpgq_kmers_read_ext")
        return out


def complete_prefix(buf, at_eof=False):
    """hpgq_fastq_complete_prefix: bytes of `buf` holding whole FASTQ records."""
    return int(lib.hpgq_fastq_complete_prefix(buf, len(buf), 1 if at_eof else 0))


class Parser:
    """hpgq_parser: FASTQ text -> device batch (parsing half of fastq_fread_se,
    src/stats_fastq.c:183, on the GPU)."""

    def __init__(self, device=0, stream=None):
        h = C.c_void_p()
        check(lib.hpgq_parser_open(C.byref(h), device, stream), "hpgq_parser_open")
        self._h = h
        self.num_reads = 0

    def close(self):
        if self._h:
            lib.hpgq_parser_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def parse(self, text):
        """Host bytes (whole records) -> device Batch (valid until the next parse)."""
        b = Batch()
        check(lib.hpgq_parse_host(self._h, text, len(text), C.byref(b)), "hpgq_parse_host")
        self.num_reads = int(b.num_reads)
        return b

    @property
    def max_length(self):
        """The longest record of the last parse (hpgq_parser_max_length)."""
        return int(lib.hpgq_parser_max_length(self._h))

    def records(self):
        n = self.num_reads
        out = {k: np.zeros(n, np.uint32) for k in ("start", "seq", "plus", "qual")}
        check(lib.hpgq_parse_records(self._h, _ptr(out["start"]), _ptr(out["seq"]),
                                     _ptr(out["plus"]), _ptr(out["qual"])), "hpgq_parse_records")
        return out
