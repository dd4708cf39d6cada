"""CPU tests of the checker itself: the C oracle (oracle/hpgq_oracle.c) and the
pure-Python restatement (oracle/pyref.py) against the hand-derived KATs in
tests/golden/, the committed synthetic vectors (tests/golden/make_golden.py)
and each other.  No GPU."""
import json
import zlib
import os

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from fastq_io import read_fastq, check_partial
from oracle import pyref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_expected.json")))


def _pyref_params(p):
    return pyref.default_params(**p.as_dict())


def _pyref_run(p, reads, reads2=None):
    mask, trims, ctr = pyref.run(_pyref_params(p), reads.pairs(),
                                 reads2.pairs() if reads2 is not None else None)
    return (np.array(mask, np.uint8), np.array(trims, np.uint32), np.array(ctr, np.uint64))


def _kat_params(section):
    lmax = KAT["lmax"]
    if section == "stats":
        return H.stats_params(lmax=lmax)
    if section == "filter":
        return H.stats_params(lmax=lmax, **KAT["filter"]["flags"])
    return H.edit_params(lmax=lmax, stats=True, **KAT["edit"]["flags"])


@pytest.mark.parametrize("section", ["stats", "filter", "edit"])
def test_kat_c_oracle_and_pyref(section):
    reads = read_fastq(os.path.join(GOLD, KAT["reads"]))
    p = _kat_params(section)
    lay = H.layout(KAT["lmax"])
    for mask, trim, ctr in (O.run(p, reads), _pyref_run(p, reads)):
        exp = KAT[section]
        check_partial(ctr, exp, KAT["lmax"], lay)
        if "mask" in exp:
            np.testing.assert_array_equal(mask, exp["mask"])
        if "trim" in exp:
            np.testing.assert_array_equal(trim, exp["trim"])


def _signed_params(section):
    k = KAT["signed"]
    if section == "stats":
        return H.stats_params(lmax=k["lmax"])
    if section == "filter":
        return H.stats_params(lmax=k["lmax"], **k["filter"]["flags"])
    return H.edit_params(lmax=k["lmax"], stats=True, **k["edit"]["flags"])


@pytest.mark.parametrize("section", ["stats", "filter", "edit"])
def test_kat_signed_qualities(section):
    """Quality bytes >= 128 as signed `char` (src/stats_fastq.c:353-355, Q13)."""
    k = KAT["signed"]
    reads = read_fastq(os.path.join(GOLD, k["reads"]))
    p = _signed_params(section)
    lay = H.layout(k["lmax"])
    for mask, trim, ctr in (O.run(p, reads), _pyref_run(p, reads)):
        exp = k[section]
        check_partial(ctr, exp, k["lmax"], lay)
        if "mask" in exp:
            np.testing.assert_array_equal(mask, exp["mask"])
        if "trim" in exp:
            np.testing.assert_array_equal(trim, exp["trim"])


@pytest.mark.parametrize("case", ["plain", "filter"])
def test_report_golden_files(case):
    """The committed report files (tests/golden/report/) are what the
    restatement of src/stats_report.c (oracle/report_ref.py) makes of the
    pure-Python counters of their input."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mrg", os.path.join(GOLD, "make_report_golden.py"))
    mrg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrg)
    rd = read_fastq(os.path.join(GOLD, "report", mrg.FQ))
    files = mrg.expected(case, rd)
    assert len(files) == 7
    for suffix, data in files.items():
        with open(os.path.join(GOLD, "report", case, f"{mrg.FQ}.{suffix}"), "rb") as f:
            assert f.read() == data, suffix


@pytest.mark.parametrize("case", ["cgr", "cgr_k2"])
def test_kat_cgr(case):
    c = KAT[case]
    reads = read_fastq(os.path.join(GOLD, c["reads"]))
    ts, tq, wc = O.cgr(c["k"], reads, c["base_quality"])
    np.testing.assert_array_equal(ts, c["table_seq"])
    np.testing.assert_array_equal(tq, c["table_q"])
    assert int(wc[0]) == c["word_count"]
    ps, pq, pw = pyref.cgr_fill(c["k"], c["base_quality"], reads.pairs())
    assert ps == c["table_seq"] and pq == c["table_q"] and pw == c["word_count"]


def _golden_cases():
    return sorted(f for f in os.listdir(GOLD) if f.startswith("synth_") and f.endswith(".npz"))


@pytest.mark.parametrize("name", _golden_cases())
def test_committed_vectors(name):
    """C oracle reproduces the committed vectors (made by the pure-Python
    restatement, tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLD, name))   # allow_pickle stays False
    p = H.params_default(**json.loads(str(z["params"])))
    r1 = O.Reads(z["seq"], z["qual"], z["idx"])
    r2 = O.Reads(z["seq2"], z["qual2"], z["idx2"]) if p.paired else None
    if name.startswith("synth_cgr"):
        ts, tq, wc = O.cgr(int(z["k"]), r1, 33)
        np.testing.assert_array_equal(ts, z["table_seq"])
        np.testing.assert_array_equal(tq, z["table_q"])
        assert int(wc[0]) == int(z["word_count"])
        return
    mask, trim, ctr = O.run(p, r1, r2)
    np.testing.assert_array_equal(mask, z["mask"])
    np.testing.assert_array_equal(ctr, z["counters"])
    if p.edit_on:
        np.testing.assert_array_equal(trim, z["trim"])


EDGE = [(b"", b""), (b"A", b"I"), (b"acgtn", b"IIIII"), (b"RYKMSWBDHV", b"5" * 10),
        (b"ACGT", bytes([200, 150, 33, 127])), (b"N" * 40, b"#" * 40), (b"GC" * 20, b"?" * 40)]


def _random_reads(rng, n, lmax, alphabet=b"ACGTN"):
    pairs = []
    for _ in range(n):
        L = int(rng.integers(0, lmax + 3))
        s = np.array(rng.choice(list(alphabet), L), np.uint8).tobytes()
        q = rng.integers(33, 75, L).astype(np.uint8).tobytes()
        pairs.append((s, q))
    return pairs


PARAM_CASES = [
    ("stats", dict()),
    ("filter_q_len", dict(read_quality_range="20,", read_length_range="50,")),
    ("filter_all", dict(read_quality_range="15,35", read_length_range="10,120", max_N=2,
                        max_out_of_quality=5, left_length=10, left_quality_range="20,",
                        right_length=15, right_quality_range="18,40")),
    ("phred64", dict(quality_encoding="phred64", read_quality_range="0,")),
]


@pytest.mark.parametrize("name,flags", PARAM_CASES)
def test_c_oracle_matches_pyref_random(name, flags):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    lmax = 100
    pairs = _random_reads(rng, 300, lmax, b"ACGTNacg") + EDGE
    reads = O.Reads.from_pairs(pairs)
    p = H.stats_params(lmax=lmax, **flags)
    for a, b in zip(O.run(p, reads), _pyref_run(p, reads)):
        np.testing.assert_array_equal(a, b)


def test_c_oracle_matches_pyref_edit_and_pe():
    rng = np.random.default_rng(7)
    lmax = 80
    pairs = _random_reads(rng, 200, lmax)
    r1 = O.Reads.from_pairs(pairs)
    r2 = O.Reads.from_pairs(_random_reads(rng, 200, lmax))
    pe = H.edit_params(lmax=lmax, stats=True, left_length=8, left_quality_range="25,",
                       right_length=12, right_quality_range="25,", read_length_range="20,")
    for a, b in zip(O.run(pe, r1), _pyref_run(pe, r1)):
        np.testing.assert_array_equal(a, b)
    pp = H.stats_params(lmax=lmax, read_quality_range="20,", read_length_range="30,")
    pp.paired = 1
    for a, b in zip(O.run(pp, r1, r2), _pyref_run(pp, r1, r2)):
        np.testing.assert_array_equal(a, b)


def test_oracle_threads_invariant():
    reads = O.synth(20000, seed=3, L=150)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    a = O.run(p, reads, nthreads=1)
    b = O.run(p, reads, nthreads=4)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_synth_generator_host_matches_oracle():
    """hpgq_synth_indices_host (libhpgq, host code) == oracle_synth lengths."""
    import ctypes as C
    s = H.Synth(2, 150, 5, 5, 1, 33, 0)
    n = 5000
    idx = np.zeros(n + 1, np.int32)
    H.check(H.lib.hpgq_synth_indices_host(C.byref(s), 1000, n, idx.ctypes.data), "idx")
    ref = O.synth(n, seed=2, L=150, first=1000)
    np.testing.assert_array_equal(idx - idx[0], ref.idx - ref.idx[0])


def test_cgr_c_oracle_matches_pyref_random_and_homopolymers():
    rng = np.random.default_rng(11)
    pairs = _random_reads(rng, 60, 90, b"ACGTNa")
    pairs += [(b"A" * 90, b"I" * 90), (b"T" * 90, b"5" * 90), (b"ACGT" * 10 + b"A" * 30, b"?" * 70)]
    reads = O.Reads.from_pairs(pairs)
    for k in (1, 3, 5):
        ts, tq, wc = O.cgr(k, reads, 33)
        ps, pq, pw = pyref.cgr_fill(k, 33, reads.pairs())
        np.testing.assert_array_equal(ts, ps)
        np.testing.assert_array_equal(tq, pq)
        assert int(wc[0]) == pw
