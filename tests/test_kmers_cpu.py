"""--kmers oracle checks (CPU): the C restatement (oracle_kmers) against the
independent pure-Python one (oracle/pyref.py) and a hand-derived known answer.
Semantics are build-defined -> parity unpinned."""
import os
import sys

import numpy as np

import oracle_lib as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyref  # noqa: E402


def _dense(d, lmax):
    out = np.zeros((1024, max(lmax - 4, 0)), dtype=np.uint64)
    for (kid, p), c in d.items():
        out[kid, p] += c
    return out


def test_kmers_known_answer():
    reads = O.Reads.from_pairs([(b"ACGTACGT", b"IIIIIIII"), (b"AAAAAN", b"IIIIII"),
                                (b"acgtA", b"IIIII"), (b"TTTT", b"IIII")])
    got = O.kmers(reads, lmax=16)
    # ACGTA CGTAC GTACG TACGT at 0..3; AAAAA at 0; nothing else
    want = {(0b0001101100, 0): 1, (0b0110110001, 1): 1, (0b1011000110, 2): 1,
            (0b1100011011, 3): 1, (0, 0): 1}
    assert pyref.kmer_string(0b0001101100) == "ACGTA"
    np.testing.assert_array_equal(got, _dense(want, 16))
    np.testing.assert_array_equal(got, _dense(pyref.kmers(reads.pairs(), 16), 16))


def test_kmers_oracle_vs_pyref_random():
    rng = np.random.default_rng(7)
    pairs = []
    for _ in range(300):
        L = int(rng.integers(0, 40))
        s = np.array(rng.choice(list(b"ACGTACGTACGTNacgR"), L), np.uint8).tobytes()
        pairs.append((s, b"I" * L))
    reads = O.Reads.from_pairs(pairs)
    mask = (rng.random(len(pairs)) < 0.7).astype(np.uint8)
    for lmax in (1, 5, 9, 24, 64):
        np.testing.assert_array_equal(O.kmers(reads, lmax, mask),
                                      _dense(pyref.kmers(reads.pairs(), lmax, mask), lmax))


def test_kmers_string_order():
    assert [pyref.kmer_string(i) for i in (0, 1, 4, 1023)] == ["AAAAA", "AAAAC", "AAACA", "TTTTT"]
