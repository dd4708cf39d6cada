"""Restatement of the stats report files of src/stats_report.c (TEST INFRASTRUCTURE).

Builds the text of every `hpg-fastq stats` report file from a dense counter set
(include/hpgq.h layout) with the reference's C arithmetic spelled out:
`1.0f * a / b` and `100.0f * a / b` are float32 (a, b size_t converted to float),
`_normalize_quality(q, phred)` is C round() (halves away from zero) of the float
difference (:26), `%i` of a size_t prints its low 32 bits as an int, `%0.2f`
formats the float promoted to double.  Only tests/ (and the golden-file script
tests/golden/make_report_golden.py) use it; the product is
hpg-fastq_amd/host/hpgq_report.c.

Reference lines followed:
  report_summary     src/stats_report.c:60-153
  report_length      :157-180 (data file; the gnuplot image is out of scope)
  report_nt_content  :206-352 (GC histogram, GC per nt, quality per nt, nucleotides)
  report_quality     :355-390 (read quality histogram; its quality.per.nt.data is
                     overwritten by report_nt_content's, which runs later: quirk Q6)
Quirk decisions: per-position maps are read by position (Q3);
mean quality from the exact fixed-point sum of per-read means, converted to float
once (Q2); 101 GC bins, the reference's printed subset 1..99 (Q4); 256 mean-Q bins,
keys as signed char (Q5, Q13).
"""
import math

import numpy as np

from oracle import pyref

f32 = np.float32


def _fdiv(a, b):
    """C `1.0f * a / b` with a, b size_t: float32 product and quotient (0 for b = 0,
    where the reference divides by zero: an empty run, quirk Q14)."""
    return f32(f32(1.0) * f32(a)) / f32(b) if b else f32(0.0)


def _pct(a, b):
    """C `100.0f * a / b` (0 for b = 0, Q14)."""
    return f32(f32(100.0) * f32(a)) / f32(b) if b else f32(0.0)


def c_round(x):
    """C round(): halves away from zero."""
    x = float(x)
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def _norm_q(q, phred):
    """_normalize_quality (:26): round((quality) - (phred)) with a float quality."""
    return c_round(f32(q) - f32(phred))


def _i32(v):
    """`%i` of a size_t: its low 32 bits as an int."""
    v = int(v) & 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def _f2(v):
    return "%0.2f" % float(v)


def report_files(ctr, lmax, phred, base, opts):
    """{suffix: bytes} of the report files of one stats run.

    ctr: dense u64 counters (one set); opts: dict with filter_on and the option
    strings/ints the summary prints (read_length_range, read_quality_range,
    left_length, left_quality_range, right_length, right_quality_range, max_N,
    max_out_of_quality; absent = unset)."""
    lay = pyref.layout(lmax)
    c = [int(x) for x in ctr]
    hl = c[lay["hist_len"]:lay["hist_len"] + lmax + 1]
    hq = c[lay["hist_meanq"]:lay["hist_meanq"] + pyref.MEANQ_BINS]
    hg = c[lay["hist_gc"]:lay["hist_gc"] + pyref.GC_BINS]
    # per-position quality sums are signed (Q13): two's complement -> int before
    # the float conversion (the reference's size_t of a negative int sum would
    # overflow the int result of round(), which has no defined value)
    pq = [x - (1 << 64) if x >= 1 << 63 else x for x in c[lay["pos_qsum"]:lay["pos_qsum"] + lmax]]
    pb = {b: c[lay["pos_" + b]:lay["pos_" + b] + lmax] for b in pyref.BASES}
    num_reads = c[pyref.S_NUM_STATS]
    passed, failed = c[pyref.S_NUM_PASSED], c[pyref.S_NUM_FAILED]
    lengths = [L for L in range(lmax + 1) if hl[L]]
    min_len = lengths[0] if lengths else 0
    max_len = lengths[-1] if lengths else 0
    acc_len = sum(L * hl[L] for L in range(lmax + 1))
    tot = {b: sum(pb[b]) for b in pyref.BASES}
    nt = sum(tot.values())
    cnt = [0] * (lmax + 1)   # reads covering position j
    for j in range(lmax - 1, -1, -1):
        cnt[j] = cnt[j + 1] + hl[j + 1]
    out = {}

    # ---- report_summary (:60-153) ----
    s = ["-----------------------------------\n", "      FastQ quality report\n",
         "-----------------------------------\n", "FastQ filename: %s\n" % base, "\n"]
    if opts.get("filter_on"):
        s.append("Filter options:\n")
        if opts.get("read_length_range"):
            s.append("\tRead length range   : %s\n" % opts["read_length_range"])
        if opts.get("read_quality_range"):
            s.append("\tRead quality range  : %s\n" % opts["read_quality_range"])
        if opts.get("left_length", 0) != 0 and opts.get("left_quality_range"):
            s.append("\tLeft length         : %i nucleotides\n" % opts["left_length"])
            s.append("\tLeft quality range  : %s\n" % opts["left_quality_range"])
        if opts.get("right_length", 0) != 0 and opts.get("right_quality_range"):
            s.append("\tRight length        : %i nucleotides\n" % opts["right_length"])
            s.append("\tRight quality range : %s\n" % opts["right_quality_range"])
        if opts.get("max_N", 100000) != 100000:
            s.append("\tMax. number of Ns   : %i\n" % opts["max_N"])
        if opts.get("max_out_of_quality", 100000) != 100000 and opts.get("read_quality_range"):
            s.append("\tMax. out of quality : %i nucletotides\n" % opts["max_out_of_quality"])
        s.append("\n")
        s.append("Number of reads in file  : %d\n" % (passed + failed))
        s.append("Number of processed reads: %d (%s %%)\n" % (num_reads, _f2(_pct(num_reads, passed + failed))))
    else:
        s.append("Filter         : Disabled\n")
        s.append("Number of reads: %d\n" % num_reads)
    s.append("\n")
    s.append("Read length (min., mean, max.): (%i, %s, %i)\n" % (min_len, _f2(_fdiv(acc_len, num_reads)), max_len))
    s.append("\n")
    # acc_quality: the exact sum of per-read raw means (fixed point, two's
    # complement), converted to float once (quirk Q2)
    fx = c[pyref.S_ACC_MEANQ_FX16]
    fx = fx - (1 << 64) if fx >= 1 << 63 else fx
    acc_q = f32(fx / 65536.0)
    qual = c_round((f32(f32(1.0) * acc_q) / f32(num_reads) if num_reads else f32(0.0)) - f32(phred))
    s.append("Mean quality = %i [%c]\n" % (qual, chr((qual + phred) & 0xFF)))
    s.append("\n")
    s.append("Nucleotide content (A, C, G, T, N)\n")
    for b in "ATGCN":
        s.append("\t%s: %s %%\n" % (b, _f2(_pct(tot[b], nt))))
    s.append("GC content\n")
    s.append("\tCG: %s %%\n" % _f2(_pct(tot["G"] + tot["C"], nt)))
    s.append("\n")
    s.append("Mean quality per nucleotide position\n")
    for k in range(max_len):
        q = _norm_q(_fdiv(pq[k], cnt[k]), phred)
        s.append("\tpos. %i: %i [%c]\t" % (k + 1, q, chr((q + phred) & 0xFF)))
        if (k + 1) % 5 == 0:
            s.append("\n")
    s.append("\n")
    out["summary.txt"] = "".join(s).encode("latin-1")

    # ---- report_length (:157-180) ----
    out["length.histogram.data"] = "".join(
        "%i\t%i\n" % (i, _i32(hl[i])) for i in range(1, max_len + 1)).encode()

    # ---- report_quality (:355-390): keys are signed (bin = key & 255) ----
    # rows min_qual..max_qual with max_qual starting at 0 (:410): all-negative
    # keys still run up to key 0
    keys = [(b - 256 if b >= 128 else b) for b in range(pyref.MEANQ_BINS) if hq[b]]
    lines = []
    if keys:
        for key in range(min(keys), max(max(keys), 0) + 1):
            lines.append("%i\t%i\n" % (key - phred, _i32(hq[key & 255])))
    out["read.quality.histogram.data"] = "".join(lines).encode()

    # ---- report_nt_content (:206-352) ----
    out["GC.histogram.data"] = "".join(
        "%i\t%i\n" % (i, _i32(hg[i])) for i in range(1, 100) if hg[i]).encode()
    lines = []
    for k in range(max_len):
        t = sum(pb[b][k] for b in pyref.BASES)
        v = _pct(pb["G"][k] + pb["C"][k], t)
        if v > f32(1.0):
            lines.append("%i\t%s\n" % (k + 1, _f2(v)))
    out["GC.per.nt.data"] = "".join(lines).encode()
    out["quality.per.nt.data"] = "".join(
        "%i\t%i\n" % (k, _norm_q(_fdiv(pq[k], cnt[k]), phred)) for k in range(max_len)).encode()
    lines = []
    for k in range(max_len):
        t = sum(pb[b][k] for b in pyref.BASES)
        lines.append("%i\t%s\n" % (k + 1, "\t".join(_f2(_pct(pb[b][k], t)) for b in "ATGCN")))
    out["nucleotides.data"] = "".join(lines).encode()
    return out
