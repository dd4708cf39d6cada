"""--kmers parity: hpgq_kmers_* (gfx950) vs the oracle's 5-mer counts, bit for
bit (build-defined semantics, DESIGN.md §2.5 -> parity unpinned)."""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _dev(reads, mask=None, offset=0):
    import torch
    dev = torch.device("cuda", 0)
    pad = np.zeros(H.DEVICE_SLACK, np.uint8)
    lead = np.full(offset, ord("A"), np.uint8)
    t = dict(seq=torch.from_numpy(np.concatenate([lead, reads.seq, pad])).to(dev),
             qual=torch.from_numpy(np.concatenate([lead, reads.qual, pad])).to(dev),
             idx=torch.from_numpy((reads.idx + offset).astype(np.int32)).to(dev))
    if mask is not None:
        t["mask"] = torch.from_numpy(mask).to(dev)
    torch.cuda.synchronize()
    return t


def gpu_kmers(lmax, batches, masks=None, offset=0):
    km = H.Kmers(lmax)
    keep = []
    for i, reads in enumerate(batches):
        m = masks[i] if masks is not None else None
        t = _dev(reads, m, offset)
        keep.append(t)
        b = H.engine.device_batch(reads.n, t["seq"].data_ptr(), t["qual"].data_ptr(),
                                  t["idx"].data_ptr())
        km.count_device(b, t["mask"].data_ptr() if m is not None else None)
    km.sync()
    out = km.by_pos()
    km.close()
    return out


def _random_reads(rng, n, lo, hi, alphabet=b"ACGTACGTACGTNacgtRY"):
    pairs = []
    for _ in range(n):
        L = int(rng.integers(lo, hi))
        s = np.array(rng.choice(list(alphabet), L), np.uint8).tobytes()
        pairs.append((s, b"I" * L))
    return O.Reads.from_pairs(pairs)


@pytest.mark.parametrize("lmax", [5, 6, 20, 150, 256])
def test_kmers_edge_lengths(lmax):
    rng = np.random.default_rng(lmax)
    reads = _random_reads(rng, 3000, 0, lmax + 40)   # includes reads longer than lmax
    np.testing.assert_array_equal(gpu_kmers(lmax, [reads]), O.kmers(reads, lmax))


def test_kmers_mask_multi_batch_and_offsets():
    rng = np.random.default_rng(3)
    batches = [_random_reads(rng, 2000, 0, 160) for _ in range(3)]
    masks = [(rng.random(b.n) < 0.6).astype(np.uint8) for b in batches]
    want = np.zeros((1024, 146), dtype=np.uint64)
    for b, m in zip(batches, masks):
        O.kmers(b, 150, m, want)
    np.testing.assert_array_equal(gpu_kmers(150, batches, masks, offset=13), want)


def test_kmers_large_synthetic():
    reads = O.synth(200_000, seed=2, L=150)
    np.testing.assert_array_equal(gpu_kmers(150, [reads]), O.kmers(reads, 150))


def test_kmers_small_lmax_is_empty():
    reads = O.Reads.from_pairs([(b"ACGTACGT", b"IIIIIIII")])
    assert gpu_kmers(4, [reads]).size == 0


@pytest.mark.parametrize("case", range(24))
def test_kmers_random_combinations(case):
    """Seeded draws of lmax (5..1024), 1-3 batches, with or without a pass
    mask, leading offsets and homopolymer-heavy or odd-byte alphabets."""
    rng = np.random.default_rng(700 + case)
    lmax = int(rng.choice([5, 9, 64, 150, 156, 157, 160, 250, 252, 300, 1024]))
    alphabet = [b"ACGTACGTACGTNacgtRY", b"AAAAAAAAAAAAAAAACGTN", b"ACGT", b"ACGTN-*."][case % 4]
    batches = [_random_reads(rng, int(rng.integers(1, 1500)), 0, lmax + int(rng.integers(1, 60)),
                             alphabet) for _ in range(int(rng.integers(1, 4)))]
    masks = [(rng.random(b.n) < 0.7).astype(np.uint8) for b in batches] if case % 3 else None
    want = np.zeros((1024, max(lmax - 4, 0)), dtype=np.uint64)
    for i, b in enumerate(batches):
        O.kmers(b, lmax, masks[i] if masks else None, want)
    got = gpu_kmers(lmax, batches, masks, offset=int(rng.integers(0, 40)))
    np.testing.assert_array_equal(got, want)


def test_kmers_lmax1024_short_reads_and_empty_masks():
    """The CLI's --lmax 1024 on 150 bp reads (the tiles past the longest counted
    read idle), a batch whose reads are all masked out and one of reads
    shorter than a 5-mer (no tile at all), then a long-read batch on the same
    counters: every tile still adds exactly once."""
    rng = np.random.default_rng(11)
    short = O.synth(50_000, seed=3, L=150)
    masked = _random_reads(rng, 500, 0, 900)
    tiny = _random_reads(rng, 700, 0, 4)
    long_ = _random_reads(rng, 900, 500, 1100)
    batches = [short, masked, tiny, long_]
    masks = [np.ones(short.n, np.uint8), np.zeros(masked.n, np.uint8), np.ones(tiny.n, np.uint8),
             (rng.random(long_.n) < 0.5).astype(np.uint8)]
    want = np.zeros((1024, 1020), dtype=np.uint64)
    for b, m in zip(batches, masks):
        O.kmers(b, 1024, m, want)
    np.testing.assert_array_equal(gpu_kmers(1024, batches, masks), want)


def test_kmers_many_groups_per_workgroup():
    """More read groups than workgroups: each workgroup's tile walks several
    groups of its class (2.5 M reads, lmax 150)."""
    reads = O.synth(2_500_000, seed=4, L=150)
    np.testing.assert_array_equal(gpu_kmers(150, [reads]), O.kmers(reads, 150))
