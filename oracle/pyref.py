"""Pure-Python restatement of the hpg-fastq QC hot path (TEST INFRASTRUCTURE).

A second, independent restatement of the rules in oracle/hpgq_oracle.c, written
as plain loops so it reads like the reference C.  It exists to cross-check the
C oracle on the small hand-written fixtures in tests/golden/ (it is far too
slow for anything bigger).  Only tests/ import it.

Parity status: "parity unpinned" — see oracle/hpgq_oracle.c and DESIGN.md §3.
Reference lines followed:
  consumer merge      src/stats_fastq.c:257-417
  filter options      src/filter_fastq.c:140-145, src/stats_options.c:275-282
  edit options        src/edit_fastq.c:148-151, src/edit_options.c:280-283
  chaos game          old/chaos_game.c:165-267
  --kmers merge       src/stats_fastq.c:384-410 (per-read k-mers: build-defined)
  CGR post-processing old/chaos_game.c:269-593 (cgr_* below; C float/double/int
                      conversions spelled out with numpy scalars)
"""

NUM_SCALARS = 8
S_NUM_INPUT, S_NUM_PASSED, S_NUM_FAILED, S_NUM_EDITED = 0, 1, 2, 3
S_NUM_STATS, S_ACC_MEANQ_FX16, S_LONG_READS = 4, 5, 6
MEANQ_BINS, GC_BINS = 256, 101
BASES = "ACGTN"


def layout(lmax):
    """Offsets of the packed counter set (include/hpgq.h)."""
    o = {"hist_len": NUM_SCALARS}
    o["hist_meanq"] = o["hist_len"] + lmax + 1
    o["hist_gc"] = o["hist_meanq"] + MEANQ_BINS
    o["pos_qsum"] = o["hist_gc"] + GC_BINS
    for i, b in enumerate(BASES):
        o["pos_" + b] = o["pos_qsum"] + lmax * (1 + i)
    o["len"] = o["pos_qsum"] + lmax * 6
    return o


def sq(c):
    """A quality byte as the reference's `char` (signed on x86-64 gcc): the
    merge adds fq_read->quality[j] into an int, src/stats_fastq.c:353-355
    (DESIGN.md §2.3, quirk Q13).  Every quality rule uses this value."""
    return c - 256 if c >= 128 else c


def c_round_div(s, n):
    """C round(s / n) for n > 0: halves away from zero."""
    return (2 * s + n) // (2 * n) if s >= 0 else -((-2 * s + n) // (2 * n))


def default_params(**kw):
    p = dict(phred=33, lmax=256, stats_on=1, filter_on=0, edit_on=0, paired=0,
             min_read_length=0, max_read_length=100000,
             min_read_quality=0, max_read_quality=100000,
             max_out_of_quality=100000,
             left_length=0, min_left_quality=0, max_left_quality=100000,
             right_length=0, min_right_quality=0, max_right_quality=100000,
             max_N=100000,
             edit_left_length=0, edit_min_left_quality=0, edit_max_left_quality=100000,
             edit_right_length=0, edit_min_right_quality=0, edit_max_right_quality=100000)
    p.update(kw)
    return p


def trim(p, q):
    """fastq_edit, build-defined leading/trailing out-of-range run trim."""
    n = len(q)
    ts = te = 0
    if p["edit_left_length"] > 0:
        lim = min(p["edit_left_length"], n)
        while ts < lim:
            Q = sq(q[ts]) - p["phred"]
            if p["edit_min_left_quality"] <= Q <= p["edit_max_left_quality"]:
                break
            ts += 1
    if p["edit_right_length"] > 0:
        lim = min(p["edit_right_length"], n - ts)
        while te < lim:
            Q = sq(q[n - 1 - te]) - p["phred"]
            if p["edit_min_right_quality"] <= Q <= p["edit_max_right_quality"]:
                break
            te += 1
    return ts, te


def passes(p, s, q):
    """fastq_filter, build-defined (Phred thresholds, exact-integer means)."""
    n = len(s)
    if n < p["min_read_length"] or n > p["max_read_length"]:
        return False
    Q = [sq(c) - p["phred"] for c in q]
    if sum(1 for c in s if c == ord("N")) > p["max_N"]:
        return False
    tot = sum(Q)
    if not (p["min_read_quality"] * n <= tot <= p["max_read_quality"] * n):
        return False
    oor = sum(1 for x in Q if x < p["min_read_quality"] or x > p["max_read_quality"])
    if oor > p["max_out_of_quality"]:
        return False
    if p["left_length"] > 0:
        k = min(p["left_length"], n)
        sl = sum(Q[:k])
        if k > 0 and not (p["min_left_quality"] * k <= sl <= p["max_left_quality"] * k):
            return False
    if p["right_length"] > 0:
        k = min(p["right_length"], n)
        sr = sum(Q[n - k:])
        if k > 0 and not (p["min_right_quality"] * k <= sr <= p["max_right_quality"] * k):
            return False
    return True


def merge(c, lay, lmax, s, q):
    """Consumer merge of one read, src/stats_fastq.c:283-382 (no length cap
    there; this dense set keeps lengths <= lmax and positions < lmax, and a
    longer read counts in S_LONG_READS and merges everything else)."""
    n = len(s)
    c[S_NUM_STATS] += 1
    if n > lmax:
        c[S_LONG_READS] += 1
    else:
        c[lay["hist_len"] + n] += 1
    gc = 0
    for j in range(n):
        ch = chr(s[j])
        if ch in "GC":
            gc += 1
        if j >= lmax:
            continue
        c[lay["pos_qsum"] + j] += sq(q[j])
        if ch in BASES:
            c[lay["pos_" + ch] + j] += 1
    if n > 0:
        sraw = sum(sq(x) for x in q)
        c[lay["hist_meanq"] + (c_round_div(sraw, n) & 255)] += 1
        c[lay["hist_gc"] + (100 * gc) // n] += 1
        c[S_ACC_MEANQ_FX16] += (sraw << 16) // n


def run(p, reads, reads2=None):
    """reads: list of (seq bytes, qual bytes).  Returns (mask, trims, counters)."""
    lmax = p["lmax"]
    lay = layout(lmax)
    nsets = 2 if p["paired"] else 1
    sets = [[0] * lay["len"] for _ in range(nsets)]
    mask, trims = [], []
    trims2 = []
    for i, (s, q) in enumerate(reads):
        mates = [(s, q)] + ([reads2[i]] if p["paired"] else [])
        evals = []
        for (ms, mq) in mates:
            ts, te = trim(p, mq) if p["edit_on"] else (0, 0)
            ws, wq = ms[ts:len(ms) - te], mq[ts:len(mq) - te]
            ok = passes(p, ws, wq) if p["filter_on"] else True
            evals.append((ts, te, ws, wq, ok))
        ok = all(e[4] for e in evals)
        mask.append(1 if ok else 0)
        trims.append(evals[0][0] | (evals[0][1] << 16))
        if p["paired"]:
            trims2.append(evals[1][0] | (evals[1][1] << 16))
        for m, (ts, te, ws, wq, _) in enumerate(evals):
            c = sets[m]
            c[S_NUM_INPUT] += 1
            c[S_NUM_PASSED if ok else S_NUM_FAILED] += 1
            if ts + te > 0:
                c[S_NUM_EDITED] += 1
            if p["stats_on"] and ok:
                merge(c, lay, lmax, ws, wq)
    out = [x & 0xFFFFFFFFFFFFFFFF for st in sets for x in st]   # u64 wrap
    return mask, trims + trims2, out


def cgr_fill(k, base_quality, reads, status=None, only_valid=False,
             table_seq=None, table_q=None, word_count=0):
    """chaos_game_fill_tables, old/chaos_game.c:165-267 (one call = one batch)."""
    dim = 1 << k
    M = 0xFFFFFFFF
    if table_seq is None:
        table_seq = [0] * (dim * dim)
        table_q = [0] * (dim * dim)
    sub = base_quality * k
    fx = fy = float(dim * 0.5)
    cnt = 0
    acc = 0
    for i, (s, q) in enumerate(reads):
        if only_valid and (status is None or status[i] != 1):
            continue
        qs = [c - 256 if c >= 128 else c for c in q]   # signed char
        for j in range(len(s)):
            qc = qs[j]
            b = s[j]
            if b == 65:
                fx = fx + ((dim - fx) * 0.5); fy = fy * 0.5
                cnt += 1; acc = (acc + qc) & M
            elif b == 67:
                fx = fx * 0.5; fy = fy * 0.5
                cnt += 1; acc = (acc + qc) & M
            elif b == 71:
                fx = fx * 0.5; fy = fy + ((dim - fy) * 0.5)
                cnt += 1; acc = (acc + qc) & M
            elif b == 84:
                fx = fx + ((dim - fx) * 0.5); fy = fy + ((dim - fy) * 0.5)
                cnt += 1; acc = (acc + qc) & M
            elif b == 78:
                cnt = 0; acc = 0
            if cnt == k:
                cx, cy = int(fx), int(fy)
                if cx == dim:
                    cx = dim - 1; fx = fx - 0.00001
                if cy == dim:
                    cy = dim - 1; fy = fy - 0.00001
                table_seq[cx * dim + cy] = (table_seq[cx * dim + cy] + 1) & M
                word_count = (word_count + 1) & M
                cnt -= 1
                table_q[cx * dim + cy] = (table_q[cx * dim + cy] + acc - sub) & M
                acc = (acc - qs[j + 1 - k]) & M
        cnt = 0
        acc = 0
    return table_seq, table_q, word_count


def kmers(reads, lmax, mask=None):
    """stats --kmers, build-defined: {(kmer id, start pos): count}."""
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    out = {}
    for r, (s, _q) in enumerate(reads):
        if mask is not None and mask[r] != 1:
            continue
        s = s.decode("latin-1") if isinstance(s, bytes) else s
        for p in range(len(s) - 4):
            if p >= lmax - 4:
                break
            word = s[p:p + 5]
            if all(ch in code for ch in word):
                kid = 0
                for ch in word:
                    kid = kid * 4 + code[ch]
                out[(kid, p)] = out.get((kid, p), 0) + 1
    return out


def kmer_string(kid):
    """id -> 5 letters, first base most significant (kmers_string, src/stats_fastq.c:479)."""
    return "".join("ACGT"[(kid >> (2 * (4 - i))) & 3] for i in range(5))


# ---- CGR post-processing (old/chaos_game.c:269-593) -------------------------
GS_HEADER_BYTES = 196   # header_gs_t, old/chaos_game.h:65-70


def cgr_gs_bytes(table, k, word_count, name=b""):
    """A GS file: header_gs_t {char[180], k, dim_x, dim_y, ref_word_count} + u32 table."""
    import struct
    dim = 1 << k
    return (name[:179].ljust(180, b"\0") + struct.pack("<4I", k, dim, dim, word_count) +
            b"".join(struct.pack("<I", int(v) & 0xFFFFFFFF) for v in table))


def cgr_table_dif(k, table_seq, fq_words, table_gs, ref_words):
    """chaos_game_calculate_table_dif (:320-373): int(seq*fq_norm - gs*gs_norm)."""
    mem = 1 << (2 * k)
    fq_norm = 128.0 / (1.0 * fq_words / mem)
    gs_norm = 128.0 / (1.0 * ref_words / mem)
    dif = [int(float(a) * fq_norm - float(b) * gs_norm) for a, b in zip(table_seq, table_gs)]
    hi, lo = -32768, 32768   # (:342-343)
    for v in dif:
        hi = max(hi, v)
        lo = min(lo, v)
    return dif, hi, lo


def cgr_dif_stats(table_dif):
    """chaos_game_validate_table_dif (:375-408), accumulators zeroed (quirk Q12)."""
    n = float(len(table_dif))
    m = 0.0
    for v in table_dif:
        m += v
    m /= n
    s = 0.0
    for v in table_dif:
        s += (v - m) ** 2
    return m, (s / n) ** 0.5


def cgr_normalize_quality(k, table_seq, table_q):
    """chaos_game_normalize_quality_table_ (:487-502): q / k / count (unsigned division)."""
    return [(q // k) // c if c > 0 else 0 for c, q in zip(table_seq, table_q)]


def cgr_pgm(k, table, norm):
    """chaos_game_generate_pgm_file_ (:521-593): bytes of the binary PGM."""
    import numpy as np
    dim = 1 << k
    redim = 128 if k < 7 else dim
    zoom = 1 << (7 - k) if k < 7 else 1
    img = bytearray(redim * redim)
    for i in range(dim):
        for j in range(dim):
            v = np.float32(np.float32(table[i * dim + j]) * np.float64(norm))   # float * double -> float
            px = int(v) & 0xFF                                                      # (int), then (uchar)
            for ii in range(zoom):
                for jj in range(zoom):
                    img[(i * zoom + ii) * redim + j * zoom + jj] = px
    return b"P5\n%d %d\n255\n" % (redim, redim) + bytes(img)
