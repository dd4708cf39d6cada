"""ASan + UBSan builds of the host code, CPU only:
  * the CPU oracle driven on edge cases (tests/sanitize/oracle_main.c);
  * the C host's option parser and report writer (hpg-fastq_amd/host/
    hpgq_options.c, hpgq_report.c) fed counter sets without a GPU
    (tests/sanitize/report_main.c), whose files must equal, byte for byte,
    the restatement of src/stats_report.c (oracle/report_ref.py) and the
    committed golden set tests/golden/report/.
The GPU pipeline threads are exercised by tests/test_cli_gpu.py."""
import importlib.util
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from fastq_io import read_fastq
from oracle import pyref, report_ref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def san(tmp_path_factory):
    out = tmp_path_factory.mktemp("san")
    r = subprocess.run(["make", "-C", os.path.join(HERE, "sanitize"), f"OUT={out}"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return out


def test_oracle_under_asan_ubsan(san):
    r = subprocess.run([str(san / "oracle_main")], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0 and "oracle_main: ok" in r.stdout, r.stdout + r.stderr


def _report(san, tmp, ctr, lmax, flags, name="in.fq"):
    cb = tmp / "ctr.bin"
    np.asarray(ctr, np.uint64).tofile(cb)
    fq = tmp / name
    if not fq.exists():
        fq.write_bytes(b"@r\nA\n+\nI\n")
    out = tmp / "out"
    out.mkdir(exist_ok=True)
    r = subprocess.run([str(san / "report_main"), str(cb), str(lmax), "stats", "-f", str(fq), "-o", str(out),
                        *map(str, flags)], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout + r.stderr
    return out


CASES = {
    "stats": ([], {}, {"filter_on": False}),
    "c2": (["--read-quality-range", "20,", "--read-length-range", "50,"],
           dict(read_quality_range="20,", read_length_range="50,"),
           {"filter_on": True, "read_quality_range": "20,", "read_length_range": "50,"}),
    "all": (["--read-quality-range", "15,38", "--read-length-range", "30,140", "--max-N", "2",
             "--max-out-of-quality", "20", "--left-length", "8", "--left-quality-range", "20,",
             "--right-length", "12", "--right-quality-range", "10,"],
            dict(read_quality_range="15,38", read_length_range="30,140", max_N=2, max_out_of_quality=20,
                 left_length=8, left_quality_range="20,", right_length=12, right_quality_range="10,"),
            {"filter_on": True, "read_quality_range": "15,38", "read_length_range": "30,140", "max_N": 2,
             "max_out_of_quality": 20, "left_length": 8, "left_quality_range": "20,", "right_length": 12,
             "right_quality_range": "10,"}),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("lmax", [150, 1024])
def test_report_writer_matches_restatement(san, tmp_path, case, lmax):
    flags, kw, opts = CASES[case]
    reads = O.synth(20000, seed=9, L=150, trunc_pct=20, n_per_1024=10)
    _, _, ctr = O.run(H.stats_params(lmax=lmax, **kw), reads)
    out = _report(san, tmp_path, ctr, lmax, flags)
    exp = report_ref.report_files(ctr, lmax, 33, "in.fq", opts)
    assert sorted(os.listdir(out)) == sorted(f"in.fq.{k}" for k in exp)
    for k, data in exp.items():
        assert (out / f"in.fq.{k}").read_bytes() == data, k


def test_report_writer_signed_qualities(san, tmp_path):
    """Signed mean-Q keys (Q13): bins >= 128 are negative keys in the histogram file."""
    import json
    k = json.load(open(os.path.join(GOLD, "kat_expected.json")))["signed"]
    reads = read_fastq(os.path.join(GOLD, k["reads"]))
    _, _, ctr = O.run(H.stats_params(lmax=k["lmax"]), reads)
    out = _report(san, tmp_path, ctr, k["lmax"], [])
    exp = report_ref.report_files(ctr, k["lmax"], 33, "in.fq", {"filter_on": False})
    for name, data in exp.items():
        assert (out / f"in.fq.{name}").read_bytes() == data, name
    hist = (out / "in.fq.read.quality.histogram.data").read_text().split("\n")
    assert hist[0] == f"{-128 - 33}\t1"


@pytest.mark.parametrize("case", ["plain", "filter"])
def test_report_writer_golden(san, tmp_path, case):
    """The C writer on the pure-Python counters of the golden input == the
    committed golden files."""
    spec = importlib.util.spec_from_file_location("mrg", os.path.join(GOLD, "make_report_golden.py"))
    mrg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrg)
    flags, kw, _ = mrg.CASES[case]
    rd = read_fastq(os.path.join(GOLD, "report", mrg.FQ))
    p = H.stats_params(lmax=mrg.LMAX, **kw)
    _, _, ctr = pyref.run(pyref.default_params(**p.as_dict()), rd.pairs())
    out = _report(san, tmp_path, np.array(ctr, np.uint64), mrg.LMAX, flags, name=mrg.FQ)
    want = os.path.join(GOLD, "report", case)
    for name in sorted(os.listdir(want)):
        assert (out / name).read_bytes() == open(os.path.join(want, name), "rb").read(), name


def test_report_quality_rows_run_to_key_zero(san, tmp_path):
    """src/stats_report.c:410 starts max_qual at 0, so when every
    mean-quality key is negative (raw quality bytes >= 128, signed char:
    quirk Q13) the read.quality.histogram rows still run up to key 0 (keys
    -16 .. 0 here). The C writer and the restatement agree, and the rows
    follow that rule."""
    reads = O.synth(3000, seed=4, L=150, trunc_pct=0)
    reads.qual[:] = 0xF0 + (np.arange(reads.qual.size) % 2)   # bytes 0xF0/0xF1: -16/-15 as char
    _, _, ctr = O.run(H.stats_params(lmax=150), reads)
    out = _report(san, tmp_path, ctr, 150, [])
    exp = report_ref.report_files(ctr, 150, 33, "in.fq", {"filter_on": False})
    got = (out / "in.fq.read.quality.histogram.data").read_bytes()
    assert got == exp["read.quality.histogram.data"]
    keys = [int(line.split(b"\t")[0]) + 33 for line in got.splitlines()]
    assert keys[0] < 0 and keys[-1] == 0 and keys == list(range(keys[0], 1)), keys


@pytest.mark.parametrize("mode", ["normal", "reserve", "populate", "sigbus"])
def test_mapped_writer_failure_modes(san, mode):
    """hpgq_mapout.c under ASan/UBSan, no GPU: the prefault
    windows and guarded copies produce exact files; a failed first-window
    reservation sends the pipeline to the stream writer with the files left
    empty; a prefault window the file system cannot back is HPGQ_E_IO; a store
    past the file's end (what a full file system does to a mapping) is caught
    by the SIGBUS guard as HPGQ_E_IO and the process lives on.  The hooks are
    the options struct's writer_hook (--writer-test-hook), not the environment."""
    if not os.path.isdir("/dev/shm"):
        pytest.skip("no /dev/shm (tmpfs)")
    d = tempfile.mkdtemp(dir="/dev/shm", prefix="hpgq_mapout_")
    try:
        r = subprocess.run([str(san / "mapout_main"), mode, d], capture_output=True, text=True, timeout=300, env=ENV)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    assert r.returncode == 0 and f"mapout_main: ok {mode}" in r.stdout, r.stdout + r.stderr
