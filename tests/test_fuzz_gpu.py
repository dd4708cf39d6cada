"""Random option combinations vs the CPU oracle, bit for bit (GPU).

The hand-picked cases in test_engine_gpu.py pin each knob on its own; this
file draws seeded combinations of every knob the C-ABI carries -- subcommand
(stats / filter / edit with or without stats), read length and quality ranges,
max_N, max_out_of_quality, the 5'/3' window filters, the edit windows, phred
33 / 64, single / paired-end, lmax -- over ragged reads (lengths 0 .. lmax
around every geometry boundary: 156 hex, 160 tri, 252 wide), lowercase /
IUPAC bytes and quality bytes >= 128 (signed char), split
over two calls with absolute offsets so the counters accumulate.  Masks,
trims and the packed u64 counter sets must equal oracle_run's
(oracle/hpgq_oracle.c, restating src/stats_fastq.c:257-417 and the filter /
edit spec of DESIGN §2) whichever kernel chain the options route to, with
the first geometry forced to tri / wide or the catch-all alone on some cases.
"""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu

NCASES = 192
# first stage per case: the default chain, or forced (hpgq_debug_set_route)
ROUTES = ["auto", "auto", "tri", "wide", "auto", "auto", "tri", "single"]
LMAX = [64, 150, 156, 157, 160, 200, 250, 252, 300, 1024]
BASE_LEN = [1, 20, 63, 100, 149, 150, 151, 156, 157, 160, 161, 200, 250, 252, 253, 300]


def _range(rng, lo, hi, gap=0):
    """'a,b' | 'a,' | ',b' | 'a' with lo <= a < hi and a + gap <= b."""
    a = int(rng.integers(lo, hi))
    b = int(rng.integers(a + gap, hi + gap + 1))
    return [f"{a},{b}", f"{a},", f",{b}", f"{a}"][int(rng.integers(0, 4))]


def _reads(rng, n, lmax, phred, cap):
    """n ragged reads, each at most `cap` bases long."""
    L = int(rng.choice([b for b in BASE_LEN if b <= cap] or [cap]))
    lens = np.full(n, L, dtype=np.int64)
    cut = rng.random(n) < 0.3
    lens[cut] = rng.integers(0, L + 1, int(cut.sum()))
    spread = rng.random(n) < 0.1
    lens[spread] = rng.integers(0, cap + 1, int(spread.sum()))
    lens = np.minimum(lens, cap)
    idx = np.zeros(n + 1, dtype=np.int32)
    idx[1:] = np.cumsum(lens)
    tot = int(idx[-1])
    seq = np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.choice(5, tot, p=[.24, .24, .24, .24, .04])]
    seq = seq.copy()
    odd = rng.random(tot) < 0.003
    seq[odd] = np.frombuffer(b"acgtnRYKM-.", dtype=np.uint8)[rng.integers(0, 11, int(odd.sum()))]
    qual = (phred + rng.integers(0, 46, tot)).astype(np.uint8)
    low = rng.random(n) < 0.15   # reads with a low-quality 5' or 3' stretch
    for i in np.nonzero(low)[0][:200]:
        a, b = int(idx[i]), int(idx[i + 1])
        k = min(int(rng.integers(0, 12)), b - a)
        qual[a:a + k] = phred + rng.integers(0, 15, k)
        qual[b - k:b] = phred + rng.integers(0, 15, k)
    wild = rng.random(tot) < 0.002
    qual[wild] = rng.integers(0, 256, int(wild.sum()))
    return O.Reads(seq, qual, idx)


def _params(rng):
    lmax = int(rng.choice(LMAX))
    o = {}
    if rng.random() < 0.5:
        o["quality_encoding"] = "phred64"
    if rng.random() < 0.6:
        o["read_length_range"] = _range(rng, 0, lmax // 2 + 1, lmax // 2)
    if rng.random() < 0.6:
        o["read_quality_range"] = _range(rng, 0, 26, 10)
    if rng.random() < 0.3:
        o["max_N"] = int(rng.integers(0, 6))
    if rng.random() < 0.3:
        o["max_out_of_quality"] = int(rng.integers(0, 40))
    if rng.random() < 0.35:
        o["left_length"] = int(rng.integers(1, 40))
        o["left_quality_range"] = _range(rng, 0, 26, 10)
    if rng.random() < 0.35:
        o["right_length"] = int(rng.integers(1, 40))
        o["right_quality_range"] = _range(rng, 0, 26, 10)
    cmd = ["stats", "stats", "filter", "edit", "edit_stats"][int(rng.integers(0, 5))]
    if cmd.startswith("edit") and "left_length" not in o and "right_length" not in o:
        o["left_length"] = int(rng.integers(1, 20))
        o["left_quality_range"] = _range(rng, 10, 30)
    if cmd == "filter" and not H.options.filter_on(o):
        o["read_quality_range"] = "20,"
    if cmd == "stats":
        p = H.stats_params(lmax=lmax, **o)
    elif cmd == "filter":
        p = H.filter_params(lmax=lmax, **o)
    else:
        p = H.edit_params(lmax=lmax, stats=cmd == "edit_stats", **o)
    p.paired = int(rng.random() < 0.3)
    return p, cmd, o


@pytest.mark.parametrize("case", range(NCASES))
def test_random_option_combination(case, monkeypatch):
    route = ROUTES[case % len(ROUTES)]
    monkeypatch.setattr(H.engine, "DEFAULT_ROUTE", route)   # hpgq_debug_set_route
    rng = np.random.default_rng(1000 + case)
    p, cmd, o = _params(rng)
    n = int(rng.integers(1, 6000))
    # reads of any length: up to 120 bases past lmax (the stats' long-read tail)
    cap = p.lmax + 120
    phred = p.phred
    r1 = _reads(rng, n, p.lmax, phred, cap)
    r2 = _reads(rng, n, p.lmax, phred, cap) if p.paired else None
    m_o, t_o, c_o = O.run(p, r1, r2)

    nsets = 2 if p.paired else 1
    cut = int(rng.integers(0, n + 1))
    mask = np.zeros(n, np.uint8)
    trim = np.zeros(n * nsets, np.uint32)
    with H.Engine(p) as e:
        for lo, hi in [(0, cut), (cut, n)]:
            if hi == lo:
                continue
            b = H.engine.host_batch(r1.seq, r1.qual, r1.idx[lo:hi + 1].copy())
            b2 = H.engine.host_batch(r2.seq, r2.qual, r2.idx[lo:hi + 1].copy()) if p.paired else None
            m = np.zeros(hi - lo, np.uint8)
            t = np.zeros((hi - lo) * nsets, np.uint32)
            e.run_host(b, b2, m, t)
            e.sync()
            mask[lo:hi] = m
            trim[lo:hi] = t[:hi - lo]
            if p.paired:
                trim[n + lo:n + hi] = t[hi - lo:]
        c_g = e.counters()
        ext, lmax_ext = e.counters_ext()
        chain = e.kernel_chain
    info = f"case {case} ({route}): {cmd} paired={p.paired} lmax={p.lmax} n={n} cut={cut} {o} chain={chain}"
    np.testing.assert_array_equal(mask, m_o, err_msg=info)
    if p.edit_on:
        np.testing.assert_array_equal(trim, t_o, err_msg=info)
    if not np.array_equal(c_g, c_o):
        bad = np.nonzero(c_g != c_o)[0]
        raise AssertionError(f"{info}: counters differ at {bad[:10]} gpu={c_g[bad[:10]]} "
                             f"oracle={c_o[bad[:10]]}")
    # the full-length set: the oracle at the longest merged window
    px = H.Params.from_buffer_copy(p)
    px.lmax = lmax_ext
    _, _, c_x = O.run(px, r1, r2)
    assert int(c_x[H.S_LONG_READS]) == 0, info
    np.testing.assert_array_equal(ext, c_x, err_msg=info)
