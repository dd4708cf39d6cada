"""ctypes declarations mirroring include/hpgq.h (no torch types cross it)."""
import ctypes as C
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
# HPGQ_LIB_PATH: load another build of the same C-ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("HPGQ_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "libhpgq.so")

NO_VALUE, MIN_VALUE, MAX_VALUE = -1, 0, 100000
LMAX_LIMIT = 1024
MAX_EDIT_LENGTH = 65535   # edit windows: trims are two 16-bit fields
DEVICE_SLACK = 8   # readable bytes past the data end of device seq/quality buffers
NUM_SCALARS = 8
(S_NUM_INPUT, S_NUM_PASSED, S_NUM_FAILED, S_NUM_EDITED,
 S_NUM_STATS, S_ACC_MEANQ_FX16, S_LONG_READS) = range(7)
MEANQ_BINS, GC_BINS = 256, 101
CGR_ALL_READS, CGR_ONLY_VALID_READS = 0, 1
CGR_PATH_AUTO, CGR_PATH_EXACT = 0, 1
# hpgq_debug_set_route (tests / A/B only; the library reads no environment)
ROUTE_AUTO, ROUTE_CATCH_ALL, ROUTE_FIRST_TRI, ROUTE_FIRST_HEX, ROUTE_FIRST_WIDE = range(5)
ROUTE_NO_ADAPTIVE = 0x10
ROUTES = {"auto": ROUTE_AUTO, "single": ROUTE_CATCH_ALL, "tri": ROUTE_FIRST_TRI,
          "hex": ROUTE_FIRST_HEX, "wide": ROUTE_FIRST_WIDE,
          "auto_fixed": ROUTE_AUTO | ROUTE_NO_ADAPTIVE}

ERRORS = {0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "out of memory",
          -4: "read longer than lmax (not returned since round 6)", -5: "no HIP device", -6: "RCCL error",
          -7: "invalid ctx state", -8: "malformed FASTQ text"}


class HpgqError(RuntimeError):
    def __init__(self, code, where=""):
        self.code = code
        super().__init__(f"hpgq error {code} ({ERRORS.get(code, '?')}) in {where}")


def check(rc, where=""):
    if rc != 0:
        raise HpgqError(rc, where)
    return rc


_PARAM_FIELDS = [
    "phred", "lmax", "stats_on", "filter_on", "edit_on", "paired",
    "min_read_length", "max_read_length", "min_read_quality", "max_read_quality",
    "max_out_of_quality", "left_length", "min_left_quality", "max_left_quality",
    "right_length", "min_right_quality", "max_right_quality", "max_N",
    "edit_left_length", "edit_min_left_quality", "edit_max_left_quality",
    "edit_right_length", "edit_min_right_quality", "edit_max_right_quality",
]


class Params(C.Structure):
    _fields_ = [(f, C.c_int32) for f in _PARAM_FIELDS]

    def as_dict(self):
        return {f: getattr(self, f) for f in _PARAM_FIELDS}


class Batch(C.Structure):
    _fields_ = [("num_reads", C.c_int64), ("seq", C.c_void_p), ("quality", C.c_void_p),
                ("data_indices", C.c_void_p)]


class Synth(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("read_length", C.c_int32), ("trunc_pct", C.c_int32),
                ("bad_pct", C.c_int32), ("n_per_1024", C.c_int32), ("phred", C.c_int32),
                ("mate", C.c_int32)]


class Summary(C.Structure):
    _fields_ = [("num_reads", C.c_uint64), ("num_passed", C.c_uint64),
                ("num_failed", C.c_uint64), ("num_edited", C.c_uint64),
                ("num_input", C.c_uint64), ("min_length", C.c_int32),
                ("max_length", C.c_int32), ("acc_length", C.c_uint64),
                ("mean_length", C.c_double), ("mean_quality_raw", C.c_double),
                ("num_A", C.c_uint64), ("num_C", C.c_uint64), ("num_G", C.c_uint64),
                ("num_T", C.c_uint64), ("num_N", C.c_uint64)]


def counters_len(lmax):
    return NUM_SCALARS + (lmax + 1) + MEANQ_BINS + GC_BINS + 6 * lmax


def layout(lmax):
    o = {"hist_len": NUM_SCALARS}
    o["hist_meanq"] = o["hist_len"] + lmax + 1
    o["hist_gc"] = o["hist_meanq"] + MEANQ_BINS
    o["pos_qsum"] = o["hist_gc"] + GC_BINS
    for i, b in enumerate("ACGTN"):
        o["pos_" + b] = o["pos_qsum"] + lmax * (1 + i)
    o["len"] = counters_len(lmax)
    return o


# (name, restype, argtypes) — every symbol include/hpgq.h exports
_SIGS = [
    ("hpgq_params_init", None, [C.POINTER(Params)]),
    ("hpgq_counters_summary", C.c_int, [C.c_void_p, C.c_int, C.POINTER(Summary)]),
    ("hpgq_open", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(Params)]),
    ("hpgq_close", None, [C.c_void_p]),
    ("hpgq_run_device", C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Batch),
                                  C.c_void_p, C.c_void_p]),
    ("hpgq_run_host", C.c_int, [C.c_void_p, C.POINTER(Batch), C.POINTER(Batch),
                                C.c_void_p, C.c_void_p]),
    ("hpgq_host_batch", C.c_int, [C.c_void_p, C.c_int64, C.c_size_t, C.c_size_t,
                                  C.POINTER(Batch), C.POINTER(Batch)]),
    ("hpgq_sync", C.c_int, [C.c_void_p]),
    ("hpgq_reserve_length", C.c_int, [C.c_void_p, C.c_int64]),
    ("hpgq_read_counters_ext", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int32)]),
    ("hpgq_reset", C.c_int, [C.c_void_p]),
    ("hpgq_counters_size", C.c_size_t, [C.c_void_p]),
    ("hpgq_read_counters", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("hpgq_fold", C.c_int, [C.c_void_p]),
    ("hpgq_counters_device", C.c_void_p, [C.c_void_p]),
    ("hpgq_stream", C.c_void_p, [C.c_void_p]),
    ("hpgq_comm_unique_id", C.c_int, [C.c_char_p]),
    ("hpgq_comm_init", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p]),
    ("hpgq_allreduce", C.c_int, [C.c_void_p]),
    ("hpgq_global_counters_device", C.c_void_p, [C.c_void_p]),
    ("hpgq_comm_count", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("hpgq_debug_set_route", C.c_int, [C.c_void_p, C.c_int]),
    ("hpgq_cgr_open", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int]),
    ("hpgq_cgr_close", None, [C.c_void_p]),
    ("hpgq_cgr_fill_device", C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_int]),
    ("hpgq_cgr_sync", C.c_int, [C.c_void_p]),
    ("hpgq_cgr_reset", C.c_int, [C.c_void_p]),
    ("hpgq_cgr_read", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("hpgq_cgr_stream", C.c_void_p, [C.c_void_p]),
    ("hpgq_cgr_last_replays", C.c_int64, [C.c_void_p]),
    ("hpgq_cgr_set_path", C.c_int, [C.c_void_p, C.c_int]),
    ("hpgq_cgr_last_exact", C.c_int, [C.c_void_p]),
    ("hpgq_cgr_comm_init", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p]),
    ("hpgq_cgr_allreduce", C.c_int, [C.c_void_p]),
    ("hpgq_cgr_global_device", C.c_void_p, [C.c_void_p]),
    ("hpgq_cgr_comm_count", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("hpgq_cgr_load_gs", C.c_int, [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p]),
    ("hpgq_cgr_write_gs", C.c_int, [C.c_char_p, C.c_int, C.c_void_p, C.c_uint32]),
    ("hpgq_cgr_table_dif", C.c_int, [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                     C.c_void_p, C.c_void_p, C.c_void_p]),
    ("hpgq_cgr_dif_stats", C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("hpgq_cgr_normalize_quality", C.c_int, [C.c_int, C.c_void_p, C.c_void_p]),
    ("hpgq_cgr_write_pgm", C.c_int, [C.c_char_p, C.c_int, C.c_void_p, C.c_double]),
    ("hpgq_cgr_write_images", C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.c_void_p]),
    ("hpgq_kmers_open", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_void_p]),
    ("hpgq_kmers_close", None, [C.c_void_p]),
    ("hpgq_kmers_count_device", C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_void_p]),
    ("hpgq_kmers_sync", C.c_int, [C.c_void_p]),
    ("hpgq_kmers_reset", C.c_int, [C.c_void_p]),
    ("hpgq_kmers_size", C.c_size_t, [C.c_void_p]),
    ("hpgq_kmers_read", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("hpgq_kmers_device", C.c_void_p, [C.c_void_p]),
    ("hpgq_kmers_reserve_length", C.c_int, [C.c_void_p, C.c_int64]),
    ("hpgq_kmers_read_ext", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int32)]),
    ("hpgq_synth_length", C.c_int32, [C.POINTER(Synth), C.c_int64]),
    ("hpgq_synth_indices_host", C.c_int, [C.POINTER(Synth), C.c_int64, C.c_int64, C.c_void_p]),
    ("hpgq_synth_device", C.c_int, [C.POINTER(Synth), C.c_int64, C.c_int64, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p]),
    ("hpgq_fastq_complete_prefix", C.c_int64, [C.c_char_p, C.c_int64, C.c_int]),
    ("hpgq_parser_open", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_void_p]),
    ("hpgq_parser_close", None, [C.c_void_p]),
    ("hpgq_parse_host", C.c_int, [C.c_void_p, C.c_char_p, C.c_int64, C.POINTER(Batch)]),
    ("hpgq_parse_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(Batch)]),
    ("hpgq_parse_records", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("hpgq_parser_stream", C.c_void_p, [C.c_void_p]),
    ("hpgq_parser_max_length", C.c_int64, [C.c_void_p]),
    ("hpgq_device_count", C.c_int, []),
    ("hpgq_device_numa_node", C.c_int, [C.c_int]),
    ("hpgq_strerror", C.c_char_p, [C.c_int]),
    ("hpgq_version", C.c_char_p, []),
    ("hpgq_kernel_name", C.c_char_p, [C.c_void_p]),
    ("hpgq_kernel_chain", C.c_char_p, [C.c_void_p]),
    ("hpgq_host_alloc", C.c_int, [C.POINTER(C.c_void_p), C.c_size_t]),
    ("hpgq_host_free", None, [C.c_void_p]),
    ("hpgq_device_alloc", C.c_int, [C.c_int, C.POINTER(C.c_void_p), C.c_size_t]),
    ("hpgq_device_free", None, [C.c_void_p]),
    ("hpgq_copy_to_host", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
]


def exported_symbols():
    return [s[0] for s in _SIGS]


def _load():
    # PyTorch-ROCm bundles its own libamdhip64/libhsa-runtime64 (same SONAMEs as
    # /opt/rocm's).  If libhpgq loads first, a later `import torch` maps a second
    # HIP/HSA runtime into the process and one of them cannot open the device.
    # Importing torch first makes libhpgq bind to the already-loaded runtime by
    # SONAME, so a process that uses both (bench, tests) has exactly one.
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C hpg-fastq_amd` "
                          "(the HIP engine has no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, res, args in _SIGS:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # (an older build loaded for an A/B timing run through HPGQ_LIB_PATH
            # may predate an entry point; the in-tree library must have them all,
            # tests/test_abi_cpu.py)
            if os.environ.get("HPGQ_LIB_PATH"):
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def params_default(**kw):
    p = Params()
    lib.hpgq_params_init(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, int(v))
    return p
