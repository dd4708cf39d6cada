"""Regenerate the committed report-file vectors tests/golden/report/.

Input: tests/golden/report/report_in.fq (synthetic reads from the
counter-based generator, with some lowercase bases and N runs).  Expected
output per case: the counters of the pure-Python restatement oracle/pyref.py
(src/stats_fastq.c:257-417), turned into report files by the restatement of
src/stats_report.c:60-390, oracle/report_ref.py (the reference's float
arithmetic spelled out).  tests/test_oracle_cpu.py checks the committed files
against the restatements; tests/test_cli_gpu.py compares the CLI's report
files with them byte for byte.

  python tests/golden/make_report_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "hpg-fastq_amd"), ROOT, os.path.join(ROOT, "tests")]

import hpgfastq as H  # noqa: E402
import oracle_lib as O  # noqa: E402
from fastq_io import to_fastq  # noqa: E402
from oracle import pyref, report_ref  # noqa: E402

OUT = os.path.join(HERE, "report")
FQ = "report_in.fq"
LMAX = 1024   # the CLI default

# case -> (CLI flags, hpgq params kwargs, report options)
CASES = {
    "plain": ([], {}, {"filter_on": False}),
    "filter": (["--read-quality-range", "20,", "--read-length-range", "50,", "--max-N", "4",
                "--left-length", "5", "--left-quality-range", "15,"],
               dict(read_quality_range="20,", read_length_range="50,", max_N=4, left_length=5,
                    left_quality_range="15,"),
               {"filter_on": True, "read_quality_range": "20,", "read_length_range": "50,",
                "max_N": 4, "left_length": 5, "left_quality_range": "15,"}),
}


def reads():
    r = O.synth(600, seed=41, L=120, trunc_pct=15, n_per_1024=30)
    pairs = []
    for i, (s, q) in enumerate(r.pairs()):
        if i % 37 == 5:   # a few lowercase bases (counted nowhere per position)
            s = s[:10] + s[10:14].lower() + s[14:]
        pairs.append((s, q))
    return O.Reads.from_pairs(pairs)


def expected(case, rd):
    _flags, kw, opts = CASES[case]
    p = H.stats_params(lmax=LMAX, **kw)
    _m, _t, ctr = pyref.run(pyref.default_params(**p.as_dict()), rd.pairs())
    return report_ref.report_files(ctr, LMAX, 33, FQ, opts)


def main():
    rd = reads()
    os.makedirs(OUT, exist_ok=True)
    text, _ = to_fastq(rd)
    with open(os.path.join(OUT, FQ), "wb") as f:
        f.write(text)
    for case in CASES:
        os.makedirs(os.path.join(OUT, case), exist_ok=True)
        for suffix, data in expected(case, rd).items():
            with open(os.path.join(OUT, case, f"{FQ}.{suffix}"), "wb") as f:
                f.write(data)
        print(case, "ok")


if __name__ == "__main__":
    main()
