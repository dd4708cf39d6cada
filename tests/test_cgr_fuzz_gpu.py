"""Random CGR fill sequences vs the oracle's restatement of
old/chaos_game.c:165-267, bit for bit (GPU).

Each seeded case draws k (1..12: the stream pass up to 7, the exact kernels
above), the base quality, ALL_READS or ONLY_VALID_READS with a random status
array (40 % of cases), and 1-3 fill calls (the double state restarts per call, :180-181, and
is carried across the reads of one call, :263-264) over ragged reads that mix
uniform random bases with N stretches, homopolymer / two-base runs of random
length (around the stream pass's exactness threshold of 48-k D moves,
DESIGN §4.5), lowercase / IUPAC bytes and quality bytes >= 128 -- so the gate
between the stream pass and the exact simulation is hit from both sides.
Tables and the u32 word count must equal the oracle's, and each call must
have taken the stream pass exactly when `stream_gate` says it is exact.
"""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from test_cgr_gpu import assert_cgr, stream_gate

pytestmark = pytest.mark.gpu

NCASES = 64


def _read(rng, L, odd):
    s = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)].copy()
    for _ in range(int(rng.integers(0, 3))):   # runs: one base or an alternating pair
        if L < 2:
            break
        a = int(rng.integers(0, L - 1))
        r = int(rng.integers(2, 70))
        pat = rng.choice([b"A", b"T", b"G", b"C", b"AT", b"GT", b"AC", b"N"])
        run = np.frombuffer(pat * (r // len(pat) + 1), dtype=np.uint8)[:r]
        e = min(L, a + r)
        s[a:e] = run[:e - a]
    if odd and L:
        m = rng.random(L) < 0.01
        s[m] = np.frombuffer(b"acgtnRYKM-", dtype=np.uint8)[rng.integers(0, 10, int(m.sum()))]
    return s


def _batch(rng, base_q, odd, wild_q):
    n = int(rng.integers(1, 1500))
    L0 = int(rng.choice([1, 7, 30, 100, 150, 250, 400]))
    lens = np.where(rng.random(n) < 0.2, rng.integers(0, L0 + 1, n), L0)
    pairs = []
    for L in lens:
        s = _read(rng, int(L), odd)
        q = (base_q + rng.integers(0, 45, int(L))).astype(np.uint8)
        if wild_q and L:
            w = rng.random(int(L)) < 0.005
            q[w] = rng.integers(128, 256, int(w.sum()))
        pairs.append((s.tobytes(), q.tobytes()))
    return O.Reads.from_pairs(pairs)


@pytest.mark.parametrize("case", range(NCASES))
def test_random_cgr_fills(case):
    rng = np.random.default_rng(5000 + case)
    k = int(rng.choice([1, 2, 3, 4, 5, 6, 7, 7, 7, 8, 9, 12]))
    base_q = int(rng.choice([33, 64]))
    odd = rng.random() < 0.3
    wild_q = rng.random() < 0.2
    batches = [_batch(rng, base_q, odd, wild_q) for _ in range(int(rng.integers(1, 4)))]
    kw = dict(base_quality=base_q)
    if rng.random() < 0.4:
        kw["mode"] = H.CGR_ONLY_VALID_READS
        kw["statuses"] = [(rng.random(b.n) < rng.choice([0.5, 0.8, 0.95])).astype(np.uint8) for b in batches]
    log = []
    assert_cgr(k, batches, exact_log=log, **kw)
    # the stream pass ran wherever it is exact, the exact kernels elsewhere
    st = kw.get("statuses", [None] * len(batches))
    assert log == [int(stream_gate(k, b, s, kw.get("mode", H.CGR_ALL_READS))) for b, s in zip(batches, st)]
