"""Minimal 4-line FASTQ reader for the test fixtures (tests only)."""
import numpy as np

from oracle_lib import Reads


def read_fastq(path):
    lines = open(path, "rb").read().split(b"\n")
    pairs = []
    for i in range(0, len(lines) - 3, 4):
        assert lines[i].startswith(b"@") and lines[i + 2].startswith(b"+"), (path, i)
        pairs.append((lines[i + 1], lines[i + 3]))
    return Reads.from_pairs(pairs)


def expected_counters(exp, lmax, lay):
    """Dense counter vector from the sparse KAT description (absent = 0)."""
    import hpgfastq as H
    c = np.zeros(H.counters_len(lmax), np.uint64)
    names = {"num_input": H.S_NUM_INPUT, "num_passed": H.S_NUM_PASSED,
             "num_failed": H.S_NUM_FAILED, "num_edited": H.S_NUM_EDITED,
             "num_stats": H.S_NUM_STATS, "acc_meanq_fx16": H.S_ACC_MEANQ_FX16,
             "long_reads": H.S_LONG_READS}
    for k, v in exp.get("scalars", {}).items():
        c[names[k]] = v % (1 << 64)
    for h in ("hist_len", "hist_meanq", "hist_gc"):
        for k, v in exp.get(h, {}).items():
            c[lay[h] + int(k)] = v
    for p in ("pos_qsum", "pos_A", "pos_C", "pos_G", "pos_T", "pos_N"):
        if p in exp:
            c[lay[p]:lay[p] + lmax] = np.array(exp[p], np.int64).astype(np.uint64)
    return c


def check_partial(got, exp, lmax, lay):
    """Compare only the fields the KAT section specifies."""
    import hpgfastq as H
    names = {"num_input": H.S_NUM_INPUT, "num_passed": H.S_NUM_PASSED,
             "num_failed": H.S_NUM_FAILED, "num_edited": H.S_NUM_EDITED,
             "num_stats": H.S_NUM_STATS, "acc_meanq_fx16": H.S_ACC_MEANQ_FX16,
             "long_reads": H.S_LONG_READS}
    for k, v in exp.get("scalars", {}).items():
        # (u64 counters: a negative expected value is its two's complement)
        assert int(got[names[k]]) == v % (1 << 64), (k, int(got[names[k]]), v)
    for h, n in (("hist_len", lmax + 1), ("hist_meanq", H.MEANQ_BINS), ("hist_gc", H.GC_BINS)):
        if h in exp:
            want = np.zeros(n, np.uint64)
            for k, v in exp[h].items():
                want[int(k)] = v
            np.testing.assert_array_equal(got[lay[h]:lay[h] + n], want, err_msg=h)
    for p in ("pos_qsum", "pos_A", "pos_C", "pos_G", "pos_T", "pos_N"):
        if p in exp:
            np.testing.assert_array_equal(got[lay[p]:lay[p] + lmax],
                                          np.array(exp[p], np.int64).astype(np.uint64), err_msg=p)


def to_fastq(reads, crlf=False, plus_header=False, prefix="r"):
    """Reads -> FASTQ text; returns (bytes, list of record end offsets)."""
    nl = b"\r\n" if crlf else b"\n"
    out, ends, pos = [], [], 0
    for i in range(reads.n):
        s, q = reads.read(i)
        h = f"{prefix}{i} extra:{i % 7}".encode()
        rec = b"@" + h + nl + s + nl + (b"+" + h if plus_header else b"+") + nl + q + nl
        out.append(rec)
        pos += len(rec)
        ends.append(pos)
    return b"".join(out), ends


def split_records(text):
    """Reference splitter for the tests: per-record (start, seq, plus, qual) offsets."""
    lines, starts, p = [], [], 0
    while p < len(text):
        e = text.index(b"\n", p)
        starts.append(p)
        lines.append((p, e))
        p = e + 1
    recs = []
    for i in range(0, len(lines) - 3, 4):
        recs.append((lines[i][0], lines[i + 1][0], lines[i + 2][0], lines[i + 3][0]))
    return recs
