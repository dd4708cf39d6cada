"""The C-ABI boundary without a GPU: libhpgq.so loads, exports every function
include/hpgq.h declares (and the ctypes table matches the header), and the
host-only entry points behave; compute entry points fail loudly (no CPU
fallback) when there is no device."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import hpgfastq as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hpgq.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    names = set()
    for m in re.finditer(r"^(?!static)[A-Za-z_][\w \*]*?\b(hpgq_\w+)\s*\(", txt, flags=re.M):
        names.add(m.group(1))
    return names


def test_header_declares_what_ctypes_binds():
    assert header_functions() == set(H.exported_symbols())


def test_library_exports_every_header_function():
    out = subprocess.run(["nm", "-D", "--defined-only", H.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = header_functions() - exported
    assert not missing, missing
    for name in header_functions():
        assert getattr(H.lib, name) is not None


def test_library_is_gfx950_code_object():
    blob = open(H.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_params_init_defaults_match_reference():
    """NO_VALUE -> 0 / 100000 (src/filter_fastq.c:195-206), phred33, stats on."""
    p = H.Params()
    H.lib.hpgq_params_init(C.byref(p))
    d = p.as_dict()
    assert d["phred"] == 33 and d["stats_on"] == 1 and d["filter_on"] == 0
    for k in ("max_read_length", "max_read_quality", "max_out_of_quality",
              "max_left_quality", "max_right_quality", "max_N"):
        assert d[k] == H.MAX_VALUE, k
    for k in ("min_read_length", "min_read_quality", "left_length", "right_length"):
        assert d[k] == H.MIN_VALUE, k


def test_counters_summary_host():
    lmax = 10
    lay = H.layout(lmax)
    c = np.zeros(H.counters_len(lmax), np.uint64)
    c[H.S_NUM_STATS] = 3
    c[H.S_NUM_INPUT] = 4
    c[H.S_NUM_PASSED] = 3
    c[H.S_NUM_FAILED] = 1
    c[lay["hist_len"] + 2] = 1
    c[lay["hist_len"] + 5] = 2
    c[lay["pos_A"]:lay["pos_A"] + 3] = [1, 1, 1]
    c[H.S_ACC_MEANQ_FX16] = 3 * (40 << 16)
    s = H.summary(c, lmax)
    assert s["num_reads"] == 3 and s["min_length"] == 2 and s["max_length"] == 5
    assert s["acc_length"] == 12 and s["num_A"] == 3
    assert abs(s["mean_quality_raw"] - 40.0) < 1e-12


def test_strerror_and_version():
    assert H.lib.hpgq_strerror(-4).decode()
    assert b"gfx950" in H.lib.hpgq_version()


def test_synth_length_matches_indices():
    s = H.Synth(2, 150, 5, 5, 1, 33, 0)
    idx = np.zeros(101, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), 0, 100, idx.ctypes.data), "idx")
    lens = [H.lib.hpgq_synth_length(C.byref(s), i) for i in range(100)]
    np.testing.assert_array_equal(np.diff(idx), lens)
    assert all(20 <= x <= 150 for x in lens)


def test_invalid_arguments_rejected():
    assert H.lib.hpgq_counters_summary(None, 10, None) == -1
    p = H.params_default(lmax=H.LMAX_LIMIT + 1)
    h = C.c_void_p()
    assert H.lib.hpgq_open(C.byref(h), 0, C.byref(p)) in (-1, -5)
    # an edit window past 16 bits (trims are ts | te << 16): invalid before any device call
    for f in ("edit_left_length", "edit_right_length"):
        p = H.params_default(lmax=150, edit_on=1, **{f: H.MAX_EDIT_LENGTH + 1})
        assert H.lib.hpgq_open(C.byref(h), 0, C.byref(p)) == -1
    p = H.params_default(lmax=150, edit_on=1, edit_left_length=H.MAX_EDIT_LENGTH)
    assert H.lib.hpgq_open(C.byref(h), 0, C.byref(p)) in (0, -5)
    if h.value:
        H.lib.hpgq_close(h)


def _no_gpu():
    try:
        import torch
        return not torch.cuda.is_available()
    except Exception:
        return True


@pytest.mark.skipif(not _no_gpu(), reason="checks the no-device path")
def test_open_fails_loudly_without_device():
    """No CPU fallback: opening an engine with no HIP device is an error."""
    assert H.lib.hpgq_device_count() == 0
    with pytest.raises(H.HpgqError) as e:
        H.Engine(H.stats_params(lmax=150))
    assert e.value.code == -5


def test_host_batch_keeps_its_arrays_alive():
    """hpgq_batch_t holds raw pointers: a batch built over temporaries (e.g. a
    sliced idx copy) must keep them alive, or the ABI reads freed memory."""
    import gc
    seq = np.frombuffer(b"ACGTACGT", dtype=np.uint8).copy()
    b = H.engine.host_batch(seq, seq.copy(), np.array([2, 5, 8], dtype=np.int32).copy())
    gc.collect()
    idx = (C.c_int32 * 3).from_address(b.data_indices)
    assert list(idx) == [2, 5, 8] and b.num_reads == 2


def test_library_reads_no_environment():
    """libhpgq takes no routing or tuning choice from the environment (VERDICT
    r3: HPGQ_KERNEL / HPGQ_TRI_GEO / HPGQ_ADAPTIVE moved to
    hpgq_debug_set_route): no getenv anywhere in its sources."""
    import glob
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srcs = glob.glob(os.path.join(root, "hpg-fastq_amd", "csrc", "*"))
    assert srcs
    for f in srcs:
        assert "getenv" not in open(f, errors="replace").read(), f
