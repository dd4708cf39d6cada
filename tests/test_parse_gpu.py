"""GPU FASTQ parser: text -> device batch -> engine, against the oracle on the
same reads (every counter, mask and per-record offset), plus malformed input."""
import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from fastq_io import to_fastq, split_records

pytestmark = pytest.mark.gpu


def parse_and_run(text, params):
    with H.Parser() as ps:
        with H.Engine(params) as e:
            b = ps.parse(text)
            import torch
            mask = torch.zeros(max(b.num_reads, 1), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            if b.num_reads:
                e.run_device(b, None, mask.data_ptr(), None)
            e.sync()
            return (mask.cpu().numpy()[:b.num_reads], e.counters(), ps.records(), b.num_reads)


@pytest.mark.parametrize("crlf,plus_header", [(False, False), (True, False), (False, True)])
def test_parse_synthetic_matches_oracle(crlf, plus_header):
    reads = O.synth(20000, seed=12, L=150)
    text, _ = to_fastq(reads, crlf=crlf, plus_header=plus_header)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    mask, ctr, recs, n = parse_and_run(text, p)
    assert n == reads.n
    m_o, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(mask, m_o)
    np.testing.assert_array_equal(ctr, c_o)
    ref = np.array(split_records(text), np.uint32)
    np.testing.assert_array_equal(recs["start"], ref[:, 0])
    np.testing.assert_array_equal(recs["seq"], ref[:, 1])
    np.testing.assert_array_equal(recs["plus"], ref[:, 2])
    np.testing.assert_array_equal(recs["qual"], ref[:, 3])


def test_parse_edge_records():
    pairs = [(b"", b""), (b"A", b"@"), (b"ACGTN" * 60, b"@+" * 150), (b"acgtRYK", b"IIIIIII")] * 50
    reads = O.Reads.from_pairs(pairs)
    text, _ = to_fastq(reads)
    p = H.stats_params(lmax=300)
    mask, ctr, _, n = parse_and_run(text, p)
    assert n == reads.n
    _, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(ctr, c_o)


def test_parse_empty_text():
    with H.Parser() as ps:
        b = ps.parse(b"")
        assert b.num_reads == 0


@pytest.mark.parametrize("bad", [
    b"@r\nACGT\n-\nIIII\n",          # third line not '+'
    b"@r\nACGT\n+\nIII\n",           # quality shorter than the sequence
    b"r\nACGT\n+\nIIII\n",           # header without '@'
    b"@r\nACGT\n+\nIIII\n@s\nAC\n",  # not whole records
])
def test_parse_malformed(bad):
    with H.Parser() as ps:
        with pytest.raises(H.HpgqError) as e:
            ps.parse(bad)
        assert e.value.code == -8


@pytest.mark.parametrize("tail", [b"\n", b"\n\n\n", b"\r\n", b"\r\n\r\n", b"\n" * 100])
def test_parse_trailing_blank_lines(tail):
    """A file ending in blank lines parses to the same records; a
    blank line between records stays a format error."""
    reads = O.synth(3000, seed=14, L=120)
    text, _ = to_fastq(reads, crlf=tail.startswith(b"\r"))
    p = H.stats_params(lmax=150, read_quality_range="20,")
    mask, ctr, _, n = parse_and_run(text + tail, p)
    assert n == reads.n
    m_o, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(mask, m_o)
    np.testing.assert_array_equal(ctr, c_o)
    with H.Parser() as ps:
        assert ps.parse(b"\n\n").num_reads == 0
        with pytest.raises(H.HpgqError):
            ps.parse(b"@r\nACGT\n+\nIIII\n\n@s\nAC\n+\nII\n")


@pytest.mark.parametrize("case", range(16))
def test_parse_random_records(case):
    """Seeded record sets (lengths 0..1024, odd bytes, '@' / '+' as quality
    characters, LF or CRLF, bare or repeated '+' headers) parse to the same
    records and the same engine results as the oracle on the reads."""
    rng = np.random.default_rng(900 + case)
    n = int(rng.integers(1, 3000))
    top = int(rng.choice([10, 150, 300, 1024]))   # lmax <= HPGQ_LMAX_LIMIT
    pairs = []
    for _ in range(n):
        L = int(rng.integers(0, top + 1))
        s = np.frombuffer(b"ACGTNacgtRY", np.uint8)[rng.integers(0, 11, L)].tobytes()
        q = (33 + rng.integers(0, 60, L)).astype(np.uint8).tobytes()   # includes '@' (64)
        pairs.append((s, q))
    reads = O.Reads.from_pairs(pairs)
    crlf, plus = bool(case & 1), bool(case & 2)
    text, _ = to_fastq(reads, crlf=crlf, plus_header=plus, prefix=["r", "@r", "+r", "r:"][case % 4])
    lmax = max(top, 8)
    p = H.stats_params(lmax=lmax, read_quality_range="15,", read_length_range="3,")
    mask, ctr, recs, got_n = parse_and_run(text, p)
    assert got_n == reads.n
    m_o, _, c_o = O.run(p, reads)
    np.testing.assert_array_equal(mask, m_o)
    np.testing.assert_array_equal(ctr, c_o)
    ref = np.array(split_records(text), np.uint32)
    np.testing.assert_array_equal(recs["start"], ref[:, 0])
    np.testing.assert_array_equal(recs["qual"], ref[:, 3])
