"""The C host's command line (no device): flags, defaults and errors as the
reference's option parsers (src/stats_options.c, src/filter_options.c,
src/edit_options.c), checked against the Python twins in hpgfastq.options."""
import pytest

import hpgfastq as H
from cli_lib import print_params, run_cli


def _py(params):
    return params.as_dict()


CASES = [
    ("stats", [], lambda: H.stats_params(lmax=1024)),
    ("stats", ["--read-quality-range", "20,", "--read-length-range", "50,"],
     lambda: H.stats_params(lmax=1024, read_quality_range="20,", read_length_range="50,")),
    ("stats", ["--max-N", "3", "--max-out-of-quality", "7", "--read-quality-range", "15,35",
               "--left-length", "8", "--left-quality-range", "20,", "--right-length", "9",
               "--right-quality-range", ",40", "--quality-encoding", "phred64"],
     lambda: H.stats_params(lmax=1024, max_N=3, max_out_of_quality=7, read_quality_range="15,35",
                            left_length=8, left_quality_range="20,", right_length=9,
                            right_quality_range=",40", quality_encoding="phred64")),
    ("filter", ["--read-length-range", "30,120"],
     lambda: H.filter_params(lmax=1024, read_length_range="30,120")),
    ("edit", ["--left-length", "10", "--left-quality-range", "20,", "--right-length", "30",
              "--right-quality-range", "20,"],
     lambda: H.edit_params(lmax=1024, left_length=10, left_quality_range="20,", right_length=30,
                           right_quality_range="20,")),
    ("edit", ["--left-length", "5", "--left-quality-range", "10,30", "--read-length-range", "40,"],
     lambda: H.edit_params(lmax=1024, left_length=5, left_quality_range="10,30",
                           read_length_range="40,")),
]


@pytest.mark.parametrize("cmd,flags,py", CASES)
def test_cli_params_match_python_options(cmd, flags, py):
    assert print_params(cmd, *flags) == _py(py())


@pytest.mark.parametrize("args", [
    ["stats", "--print-params", "--read-length-range", "50,20"],
    ["stats", "--print-params", "--read-quality-range", "-3,"],
    ["stats", "--print-params", "--quality-encoding", "solexa"],
    ["filter", "--print-params"],                       # nothing to filter
    ["edit", "--print-params", "--max-N", "2"],          # nothing to edit
    ["filter", "--print-params", "--kmers", "--max-N", "1"],   # --kmers is a stats flag
    ["stats", "-f", "/nonexistent.fq"],
    ["bogus"],
    # thread counts are whole integers in range (atoi took garbage as 0)
    ["filter", "--print-params", "--max-N", "1", "--copy-threads", "abc"],
    ["filter", "--print-params", "--max-N", "1", "--copy-threads", "65"],
    ["filter", "--print-params", "--max-N", "1", "--prefault-threads", "5"],
    ["filter", "--print-params", "--max-N", "1", "--prefault-threads", "2x"],
    # the writer's failure hooks are a test option (HPGQ_WRITER_TEST_HOOKS)
    ["filter", "--print-params", "--max-N", "1", "--writer-test-hook", "1"],
    # edit windows are at most 65535 bases (trims are two 16-bit fields)
    ["edit", "--print-params", "--left-length", "65536", "--left-quality-range", "20,"],
])
def test_cli_rejects(args):
    assert run_cli(args, check=False).returncode != 0


def test_cli_accepts_valid_writer_options():
    print_params("filter", "--max-N", "1", "--copy-threads", "8", "--prefault-threads", "4")
    r = run_cli(["filter", "--print-params", "--max-N", "1", "--writer-test-hook", "2"],
                env={"HPGQ_WRITER_TEST_HOOKS": "1"})
    assert r.returncode == 0


def test_cli_lmax_option():
    assert print_params("stats", "--lmax", "150")["lmax"] == 150
