"""Random flag combinations through the C host CLI (GPU): the same seeded
option draws as test_fuzz_gpu.py, spelled as the reference's command-line
flags (src/*_options.c), on synthetic FASTQ files, small or large parse units
and one or two GPU workers.  The CLI's parsed parameters must equal the Python
option twins' (`--print-params`), and its outputs must equal the oracle's:
the counter set for `stats`, passed.fq / failed.fq for `filter`, edit.fq /
failed.fq (trimmed records) for `edit`.
"""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from cli_lib import print_params, run_cli
from fastq_io import to_fastq
from test_fuzz_gpu import _params

pytestmark = pytest.mark.gpu

FLAG = {"max_N": "--max-N"}


def _flags(o):
    out = []
    for k, v in o.items():
        out += [FLAG.get(k, "--" + k.replace("_", "-")), str(v)]
    return out


@pytest.mark.parametrize("case", range(16))
def test_cli_random_flags(tmp_path, case):
    rng = np.random.default_rng(3000 + case)
    _, cmd, o = _params(rng)
    cmd = "edit" if cmd.startswith("edit") else cmd
    flags = _flags(o)
    phred = 64 if o.get("quality_encoding") == "phred64" else 33
    # the Python twin of the command's parameters (the CLI's default lmax: 1024)
    if cmd == "stats":
        p = H.stats_params(lmax=1024, **o)
    elif cmd == "filter":
        p = H.filter_params(lmax=1024, **o)
    else:
        p = H.edit_params(lmax=1024, **o)
    got_p = print_params(cmd, *flags)
    want_p = p.as_dict()
    for k, v in got_p.items():
        if k in want_p:
            assert v == want_p[k], (case, cmd, flags, k, v, want_p[k])

    L = int(rng.choice([60, 150, 250]))
    reads = O.synth(int(rng.integers(2000, 12000)), seed=50 + case, L=L, trunc_pct=25,
                    n_per_1024=8, phred=phred)
    text, _ = to_fastq(reads)
    fq = tmp_path / "in.fq"
    fq.write_bytes(text)
    out = tmp_path / "out"
    out.mkdir()
    ctr = tmp_path / "ctr.bin"
    extra = ["--chunk-mb", int(rng.choice([1, 256])), "--gpu-workers", int(rng.integers(1, 3)), "--quiet"]
    if cmd == "stats":
        extra += ["--counters-out", ctr]
    run_cli([cmd, "-f", fq, "-o", out, *flags, *extra])
    mask, trim, want = O.run(p, reads)
    info = (case, cmd, flags)
    if cmd == "stats":
        np.testing.assert_array_equal(np.fromfile(ctr, np.uint64), want, err_msg=str(info))
        return
    recs = []
    for i in range(reads.n):
        s, q = reads.read(i)
        if cmd == "edit":
            ts, te = int(trim[i]) & 0xFFFF, int(trim[i]) >> 16
            s, q = s[ts:len(s) - te], q[ts:len(q) - te]
        recs.append(b"@" + f"r{i} extra:{i % 7}".encode() + b"\n" + s + b"\n+\n" + q + b"\n")
    ok = b"".join(r for r, m in zip(recs, mask) if m)
    bad = b"".join(r for r, m in zip(recs, mask) if not m)
    assert (out / ("passed.fq" if cmd == "filter" else "edit.fq")).read_bytes() == ok, info
    assert (out / "failed.fq").read_bytes() == bad, info
