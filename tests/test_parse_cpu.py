"""Host side of the FASTQ parser: hpgq_fastq_complete_prefix (libhpgq host
code, no device) cuts a chunk at the last whole record."""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from fastq_io import to_fastq


def _reads():
    pairs = [(b"ACGT", b"IIII"), (b"", b""), (b"NNACG", b"@@@@@"), (b"A" * 50, b"@" + b"I" * 49),
             (b"GATTACA", b"+5+5+5+")]
    return O.Reads.from_pairs(pairs * 5)


@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("plus_header", [False, True])
def test_complete_prefix_every_cut(crlf, plus_header):
    text, ends = to_fastq(_reads(), crlf=crlf, plus_header=plus_header)
    ends_a = np.array([0] + ends)
    for n in range(0, len(text) + 1):
        want = int(ends_a[ends_a <= n].max())
        got = H.complete_prefix(text[:n])
        assert got == want, (n, got, want)
    assert H.complete_prefix(text, at_eof=True) == len(text)


def test_complete_prefix_synthetic_chunks():
    reads = O.synth(3000, seed=8, L=150)
    text, ends = to_fastq(reads)
    ends_a = np.array([0] + ends)
    rng = np.random.default_rng(1)
    for n in rng.integers(0, len(text), 200):
        assert H.complete_prefix(text[:n]) == int(ends_a[ends_a <= n].max())
