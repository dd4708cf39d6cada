"""The C host CLI end to end on the GPU: FASTQ file -> hpg-fastq stats |
filter | edit -> counters / output files, against the oracle on the same
reads.  Small --chunk-mb forces records to be carried across parse units."""
import os
import subprocess

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from cli_lib import CLI, run_cli
from fastq_io import to_fastq

pytestmark = pytest.mark.gpu


def _records(reads, crlf=False):
    nl = b"\r\n" if crlf else b"\n"
    out = []
    for i in range(reads.n):
        s, q = reads.read(i)
        h = f"r{i} extra:{i % 7}".encode()
        out.append((b"@" + h + nl, s, b"+" + nl, q, nl))
    return out


def _write(tmp_path, reads, crlf=False, name="in.fq"):
    text, _ = to_fastq(reads, crlf=crlf)
    path = tmp_path / name
    path.write_bytes(text)
    return str(path)


@pytest.mark.parametrize("chunk_mb", [1, 256])
def test_cli_stats_matches_oracle(tmp_path, chunk_mb):
    reads = O.synth(20000, seed=21, L=150)
    fq = _write(tmp_path, reads)
    out = tmp_path / "out"
    out.mkdir()
    ctr = tmp_path / "ctr.bin"
    run_cli(["stats", "-f", fq, "-o", out, "--read-quality-range", "20,", "--read-length-range",
             "50,", "--lmax", 150, "--chunk-mb", chunk_mb, "--counters-out", ctr, "--quiet"])
    got = np.fromfile(ctr, np.uint64)
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    _, _, want = O.run(p, reads)
    np.testing.assert_array_equal(got, want)
    summ = (out / "in.fq.summary.txt").read_text()
    assert f"Number of processed reads: {int(want[H.S_NUM_PASSED])}" in summ
    # every report file, byte for byte, as the restatement of src/stats_report.c
    # makes it from the same counters
    from oracle import report_ref
    exp = report_ref.report_files(got, 150, 33, "in.fq",
                                  {"filter_on": True, "read_quality_range": "20,",
                                   "read_length_range": "50,"})
    for suffix, data in exp.items():
        assert (out / f"in.fq.{suffix}").read_bytes() == data, suffix


@pytest.mark.parametrize("case", ["plain", "filter"])
def test_cli_report_golden(tmp_path, case):
    """`hpg-fastq stats` report files == the committed golden set
    (tests/golden/report/, made by tests/golden/make_report_golden.py from the
    restatements of src/stats_fastq.c:257-417 and src/stats_report.c:60-390),
    byte for byte."""
    import filecmp
    import importlib.util
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("mrg", os.path.join(gold, "make_report_golden.py"))
    mrg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mrg)
    flags = mrg.CASES[case][0]
    run_cli(["stats", "-f", os.path.join(gold, "report", mrg.FQ), "-o", tmp_path, *flags, "--quiet"])
    want_dir = os.path.join(gold, "report", case)
    names = sorted(os.listdir(want_dir))
    assert len(names) == 7
    for name in names:
        assert filecmp.cmp(os.path.join(want_dir, name), tmp_path / name, shallow=False), name


WRITERS = {"mmap": [], "stream": ["--stream-writer"]}
WRITER_LINE = {"mmap": "writer: mapped output files, parallel copy", "stream": "writer: one stream writer thread"}


def run_writer(args, writer):
    """run_cli with the writer choice; asserts the pipeline used that writer
    (HPGQ_TRACE=1 prints it: a failed mapping falls back to the stream writer)"""
    r = run_cli(list(args) + WRITERS[writer], env={"HPGQ_TRACE": "1"})
    assert WRITER_LINE[writer] in r.stderr, r.stderr[-2000:]
    return r


@pytest.mark.parametrize("writer", sorted(WRITERS))
@pytest.mark.parametrize("crlf", [False, True])
def test_cli_filter_outputs(tmp_path, crlf, writer):
    """passed.fq / failed.fq byte for byte, with the mapped parallel writer
    (default) and the one-thread stream writer."""
    reads = O.synth(15000, seed=22, L=150)
    fq = _write(tmp_path, reads, crlf=crlf)
    run_writer(["filter", "-f", fq, "-o", tmp_path, "--read-quality-range", "20,",
                "--read-length-range", "50,", "--max-N", "1", "--chunk-mb", 1, "--quiet"], writer)
    p = H.filter_params(lmax=1024, read_quality_range="20,", read_length_range="50,", max_N=1)
    mask, _, _ = O.run(p, reads)
    recs = [h + sq + nl + plus + q + nl for (h, sq, plus, q, nl) in _records(reads, crlf)]
    passed = b"".join(r for r, m in zip(recs, mask) if m)
    failed = b"".join(r for r, m in zip(recs, mask) if not m)
    assert (tmp_path / "passed.fq").read_bytes() == passed
    assert (tmp_path / "failed.fq").read_bytes() == failed


@pytest.mark.parametrize("writer", sorted(WRITERS))
def test_cli_edit_outputs(tmp_path, writer):
    reads = O.synth(12000, seed=24, L=150)
    fq = _write(tmp_path, reads)
    run_writer(["edit", "-f", fq, "-o", tmp_path, "--left-length", 10, "--left-quality-range", "20,",
                "--right-length", 30, "--right-quality-range", "20,", "--read-length-range", "60,",
                "--chunk-mb", 1, "--quiet"], writer)
    p = H.edit_params(lmax=1024, left_length=10, left_quality_range="20,", right_length=30,
                      right_quality_range="20,", read_length_range="60,")
    mask, trim, _ = O.run(p, reads)
    ok, bad = [], []
    for (h, s, plus, q, nl), m, t in zip(_records(reads), mask, trim):
        ts, te = int(t) & 0xFFFF, int(t) >> 16
        rec = h + s[ts:len(s) - te] + b"\n" + plus + q[ts:len(q) - te] + b"\n"
        (ok if m else bad).append(rec)
    assert (tmp_path / "edit.fq").read_bytes() == b"".join(ok)
    assert (tmp_path / "failed.fq").read_bytes() == b"".join(bad)


def _filter_expected(reads):
    p = H.filter_params(lmax=1024, read_quality_range="20,", read_length_range="50,")
    mask, _, _ = O.run(p, reads)
    recs = [h + sq + nl + plus + q + nl for (h, sq, plus, q, nl) in _records(reads)]
    return (b"".join(r for r, m in zip(recs, mask) if m), b"".join(r for r, m in zip(recs, mask) if not m))


def test_cli_writer_reservation_failure_uses_stream_writer(tmp_path):
    """The mapped writer reserves each output's first window before using the
    mapping (hpgq_mapout.c); when that fails (test hook in the options struct,
    --writer-test-hook 1) the stream writer runs and the files are exact."""
    reads = O.synth(15000, seed=31, L=150)
    fq = _write(tmp_path, reads)
    r = run_cli(["filter", "-f", fq, "-o", tmp_path, "--read-quality-range", "20,", "--read-length-range", "50,",
                 "--chunk-mb", 1, "--quiet", "--writer-test-hook", 1],
               env={"HPGQ_TRACE": "1", "HPGQ_WRITER_TEST_HOOKS": "1"})
    assert WRITER_LINE["stream"] in r.stderr, r.stderr[-2000:]
    passed, failed = _filter_expected(reads)
    assert (tmp_path / "passed.fq").read_bytes() == passed
    assert (tmp_path / "failed.fq").read_bytes() == failed


@pytest.mark.parametrize("threads", [["--prefault-threads", 2], ["--prefault-threads", 4, "--copy-threads", 3],
                                     ["--copy-threads", 1]])
def test_cli_writer_thread_options_exact(tmp_path, threads):
    """The mapped writer's thread options (prefault threads past the reserved
    first window, fewer or more copiers than --num-threads) write exactly the
    default's files (the input spans several 32 MB prefault windows)."""
    reads = O.synth(150000, seed=34, L=150)
    fq = _write(tmp_path, reads)
    r = run_cli(["filter", "-f", fq, "-o", tmp_path, "--read-quality-range", "20,", "--read-length-range", "50,",
                 "--chunk-mb", 4, "--quiet", *threads], env={"HPGQ_TRACE": "1"})
    assert WRITER_LINE["mmap"] in r.stderr, r.stderr[-2000:]
    passed, failed = _filter_expected(reads)
    assert (tmp_path / "passed.fq").read_bytes() == passed
    assert (tmp_path / "failed.fq").read_bytes() == failed


@pytest.mark.parametrize("hook", [2, 4])
def test_cli_writer_store_failure_is_io_error(tmp_path, hook):
    """A prefault window the file system cannot back (hook 2), or a store into
    a mapped page past the file's end -- what a file system filled by another
    writer does to a mapping -- (hook 4: passed.fq shrinks to 0 behind its
    mapping) ends the run with HPGQ_E_IO and exit status 1, not a SIGBUS."""
    # (hook 2 needs an input past the 32 MB first window, which is reserved up front)
    reads = O.synth(150000 if hook == 2 else 40000, seed=32, L=150)
    fq = _write(tmp_path, reads)
    r = run_cli(["filter", "-f", fq, "-o", tmp_path, "--read-quality-range", "20,", "--read-length-range", "50,",
                 "--chunk-mb", 1, "--quiet", "--writer-test-hook", hook,
                 # (the default prefaults nothing past the first window: hook 2 needs the threads)
                 *(["--prefault-threads", 2] if hook == 2 else [])], check=False,
                env={"HPGQ_TRACE": "1", "HPGQ_WRITER_TEST_HOOKS": "1"})
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])   # (a SIGBUS death would be -7)
    assert WRITER_LINE["mmap"] in r.stderr
    assert "Error: file i/o error (-9)" in r.stderr, r.stderr[-2000:]


def test_cli_writer_to_devices(tmp_path):
    """Outputs that cannot be mapped (here: symlinks to /dev/null) take the
    stream writer, and the run succeeds."""
    reads = O.synth(3000, seed=33, L=150)
    fq = _write(tmp_path, reads)
    d = tmp_path / "out"
    d.mkdir()
    for n in ("passed.fq", "failed.fq", "edit.fq"):
        os.symlink("/dev/null", d / n)
    for cmd, extra in (("filter", ["--read-quality-range", "20,"]), ("edit", ["--left-length", 10, "--left-quality-range", "20,"])):
        r = run_cli([cmd, "-f", fq, "-o", d, "--chunk-mb", 1, "--quiet", *extra], env={"HPGQ_TRACE": "1"})
        assert WRITER_LINE["stream"] in r.stderr


@pytest.mark.parametrize("writer", sorted(WRITERS))
@pytest.mark.parametrize("case", ["empty", "all_fail", "all_pass", "no_final_newline"])
def test_cli_writer_edges(tmp_path, case, writer):
    """Output files at the edges: an empty input, every read failing (empty
    passed.fq), every read passing (empty failed.fq), a file whose last line
    lacks its newline (the reader adds it); edit the same way."""
    reads = O.synth(3000, seed=31, L=150)
    text, _ = to_fastq(reads)
    if case == "empty":
        text = b""
    elif case == "no_final_newline":
        text = text[:-1]
    fq = tmp_path / "in.fq"
    fq.write_bytes(text)
    q = {"all_fail": "60,", "all_pass": "0,"}.get(case, "20,")
    for cmd in ("filter", "edit"):
        d = tmp_path / cmd
        d.mkdir()
        extra = ["--left-length", 10, "--left-quality-range", "20,"] if cmd == "edit" else []
        run_writer([cmd, "-f", fq, "-o", d, "--read-quality-range", q, "--chunk-mb", 1, "--quiet", *extra], writer)
        if cmd == "filter":
            p = H.filter_params(lmax=1024, read_quality_range=q)
        else:
            p = H.edit_params(lmax=1024, left_length=10, left_quality_range="20,", read_quality_range=q)
        mask, trim, _ = O.run(p, reads) if case != "empty" else (np.zeros(0), np.zeros(0), None)
        ok, bad = [], []
        for (h, sq, plus, qq, nl), m, t in zip(_records(reads) if case != "empty" else [], mask, trim):
            ts, te = (int(t) & 0xFFFF, int(t) >> 16) if cmd == "edit" else (0, 0)
            rec = h + sq[ts:len(sq) - te] + nl + plus + qq[ts:len(qq) - te] + nl
            (ok if m else bad).append(rec)
        # (to_fastq writes the same records as _records; the reader restores a
        # missing final newline)
        assert (d / ("passed.fq" if cmd == "filter" else "edit.fq")).read_bytes() == b"".join(ok)
        assert (d / "failed.fq").read_bytes() == b"".join(bad)
        if case == "all_fail":
            assert not ok
        if case == "all_pass":
            assert not bad


def test_cli_kat_stats(tmp_path):
    import json
    from fastq_io import check_partial
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    kat = json.load(open(os.path.join(gold, "kat_expected.json")))
    ctr = tmp_path / "ctr.bin"
    run_cli(["stats", "-f", os.path.join(gold, kat["reads"]), "-o", tmp_path, "--lmax", kat["lmax"],
             "--counters-out", ctr, "--quiet"])
    check_partial(np.fromfile(ctr, np.uint64), kat["stats"], kat["lmax"], H.layout(kat["lmax"]))


def test_cli_reads_longer_than_lmax(tmp_path):
    """--lmax only sizes the on-chip counters: 150 bp reads at --lmax 100 give
    the full-length counters (the oracle at 150) and the report over them
    (round 5 ended such a run with "read longer than lmax")."""
    reads = O.synth(3000, seed=3, L=150)
    fq = _write(tmp_path, reads)
    ctr = tmp_path / "ctr.bin"
    run_cli(["stats", "-f", fq, "-o", tmp_path, "--lmax", 100, "--counters-out", ctr, "--quiet"])
    _, _, want = O.run(H.stats_params(lmax=150), reads)
    np.testing.assert_array_equal(np.fromfile(ctr, np.uint64), want)


def test_cli_edit_length_limit(tmp_path):
    reads = O.synth(10, seed=3, L=150)
    fq = _write(tmp_path, reads)
    r = run_cli(["edit", "-f", fq, "-o", tmp_path, "--left-length", 65536, "--left-quality-range", "20,",
                 "--quiet"], check=False)
    assert r.returncode != 0 and "at most 65535" in r.stdout


@pytest.mark.parametrize("filt", [False, True])
def test_cli_stats_kmers(tmp_path, filt):
    """stats --kmers: the raw table equals the oracle's over the merged reads (the
    passed ones when filtering), and kmers.txt / kmers.per.nt.data follow it."""
    rng = np.random.default_rng(31)
    reads = O.synth(15000, seed=31, L=150)
    fq = _write(tmp_path, reads)
    out = tmp_path / "out"
    out.mkdir()
    kb = tmp_path / "k.bin"
    flags = ["--read-quality-range", "20,", "--read-length-range", "50,"] if filt else []
    run_cli(["stats", "-f", fq, "-o", out, "--kmers", "--kmers-out", kb, "--lmax", 150,
             "--chunk-mb", 1, "--quiet"] + flags)
    got = np.fromfile(kb, np.uint64).reshape(1024, 146)
    mask = None
    if filt:
        p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
        mask, _, _ = O.run(p, reads)
    want = O.kmers(reads, 150, None if mask is None else np.asarray(mask, np.uint8))
    np.testing.assert_array_equal(got, want)
    tot = want.sum(axis=1)
    order = sorted(range(1024), key=lambda i: (-int(tot[i]), i))
    names = ["".join("ACGT"[(i >> (2 * (4 - j))) & 3] for j in range(5)) for i in range(1024)]
    lines = (out / "in.fq.kmers.txt").read_text().splitlines()
    assert lines[0] == "# Sequence\tCount"
    assert lines[1:] == [f"{names[i]}\t{int(tot[i])}" for i in order]
    rows = (out / "in.fq.kmers.per.nt.data").read_text().splitlines()
    top = order[:5]
    size = max(int(np.nonzero(want[i])[0].max()) + 1 for i in top)
    assert len(rows) == size
    assert rows[0] == "1\t" + "\t".join(str(int(want[i, 0])) for i in top)
    summ = (out / "in.fq.summary.txt").read_text()
    assert "K-mers (top 20)" in summ and f"\t{names[order[0]]}\t\t{int(tot[order[0]])}" in summ
    del rng


@pytest.mark.parametrize("filtered", [False, True])
def test_cli_chaos_game(tmp_path, filtered):
    """stats --cg --k 5 --gs-filename: the device tables (one call: the file is
    one parse unit) against the oracle, then the old tool's images and the
    difference-table summary (old/chaos_game.c:320-472) against the Python
    restatement."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyref as R
    k = 5
    reads = O.synth(8000, seed=31, L=150)
    fq = _write(tmp_path, reads, name="cg.fq")
    ref = O.synth(3000, seed=32, L=200)
    rts, _rtq, rwc = O.cgr(k, ref, 33)
    gs = tmp_path / "ref.gs"
    H.cgr_write_gs(str(gs), k, rts, int(rwc[0]))
    out = tmp_path / "out"
    out.mkdir()
    args = ["stats", "-f", fq, "-o", out, "--cg", "--k", k, "--gs-filename", gs, "--lmax", 150,
            "--quiet"]
    status = None
    if filtered:
        args += ["--read-quality-range", "20,"]
        p = H.stats_params(lmax=150, read_quality_range="20,")
        status, _, _ = O.run(p, reads)
    run_cli(args)
    ts, tq, wc = O.cgr(k, reads, 33, status=status, mode=1 if filtered else 0)
    wc = int(wc[0])
    mem = 1 << (2 * k)
    assert (out / "cg.fq_k=5_FG.pgm").read_bytes() == R.cgr_pgm(k, ts.tolist(), 128.0 / (wc / mem))
    qn = R.cgr_normalize_quality(k, ts.tolist(), tq.tolist())
    assert (out / "cg.fq_k=5_QQ.pgm").read_bytes() == R.cgr_pgm(k, qn, 256.0 / 62)
    dif, hi, lo = R.cgr_table_dif(k, ts.tolist(), wc, rts.tolist(), int(rwc[0]))
    absd = [min(abs(v), 255) for v in dif]
    assert (out / "cg.fq_k=5_FG_dif.pgm").read_bytes() == R.cgr_pgm(k, absd, 1.0)
    txt = (out / "cg.fq.chaos_game.txt").read_text()
    assert f"Words read in FastQ file: {wc}" in txt
    assert f"Interval of variation of diff matrix values = [{hi}, {lo}]" in txt


# ---- multi-GPU workers and chaos-game batches -----------------
def _homopolymer_reads(n, seed):
    """Reads whose long poly-A / poly-T stretches carry the CGR double state to
    the clamp, so the tables depend on where the fill calls start."""
    rng = np.random.default_rng(seed)
    pairs = []
    for i in range(n):
        L = int(rng.integers(60, 160))
        if i % 3 == 0:
            s = (b"A" if rng.integers(2) else b"T") * L
        else:
            s = rng.choice(np.frombuffer(b"ACGTN", np.uint8), size=L,
                           p=[0.3, 0.2, 0.2, 0.29, 0.01]).tobytes()
        q = rng.integers(35, 75, size=L, dtype=np.uint8).tobytes()
        pairs.append((s, q))
    return O.Reads.from_pairs(pairs)


def _cg_batches(text_ends, reads, B):
    """Records ending in ((j-1)B, jB] form chaos-game call j (hpgq_pipeline.c)."""
    groups = {}
    for i, e in enumerate(text_ends):
        groups.setdefault((e - 1) // B, []).append(i)
    return [O.Reads.from_pairs([reads.read(i) for i in idx]) for _j, idx in sorted(groups.items())]


@pytest.mark.parametrize("chunk_mb,gpus", [(1, 1), (1, 2), (4, 3), (256, 1)])
def test_cli_cg_batches_independent_of_chunks_and_workers(tmp_path, chunk_mb, gpus):
    """--cg makes one chaos_game_fill_tables call per --cg-batch-size bytes of
    FASTQ text (records ending in ((j-1)B, jB]), whatever --chunk-mb and
    --gpus are: the tables equal the oracle's calls over those batches on an
    input whose tables depend on the call boundaries (homopolymer runs)."""
    reads = _homopolymer_reads(12000, 5)
    text, ends = to_fastq(reads)
    fq = tmp_path / "hp.fq"
    fq.write_bytes(text)
    B = 300_000
    cgo = tmp_path / "cg.bin"
    run_cli(["stats", "-f", fq, "-o", tmp_path, "--cg", "--k", 6, "--cg-batch-size", B,
             "--chunk-mb", chunk_mb, "--gpus", gpus, "--lmax", 160, "--cg-out", cgo, "--quiet"])
    got = np.fromfile(cgo, np.uint32)
    dim2 = 1 << 12
    ts, tq, wc = np.zeros(dim2, np.uint32), np.zeros(dim2, np.uint32), np.zeros(1, np.uint32)
    for b in _cg_batches(ends, reads, B):
        O.cgr(6, b, 33, tables=(ts, tq, wc))
    np.testing.assert_array_equal(got[:dim2], ts)
    np.testing.assert_array_equal(got[dim2:2 * dim2], tq)
    assert int(got[-1]) == int(wc[0])
    # and the split matters on this input: one call over everything differs
    ts1, _, _ = O.cgr(6, reads, 33)
    assert not np.array_equal(ts1, ts)


@pytest.mark.parametrize("cmd", ["stats", "filter", "edit"])
def test_cli_workers_merge(tmp_path, cmd):
    """--gpus 3 --gpu-workers 2 (six workers; on a one-GPU box they share device
    0) with small chunks: counters, k-mer tables and output files equal one
    worker's."""
    reads = O.synth(30000, seed=27, L=150, n_per_1024=6)
    fq = _write(tmp_path, reads)
    outs = []
    for g in (1, 3):
        d = tmp_path / f"g{g}"
        d.mkdir()
        args = [cmd, "-f", fq, "-o", d, "--chunk-mb", 1, "--gpus", g, "--gpu-workers", 1 if g == 1 else 2,
                "--counters-out", d / "ctr.bin",
                "--quiet", "--read-quality-range", "20,", "--read-length-range", "50,"]
        if cmd == "stats":
            args += ["--kmers", "--kmers-out", d / "km.bin", "--lmax", 150]
        if cmd == "edit":
            args += ["--left-length", 10, "--left-quality-range", "20,"]
        run_cli(args)
        outs.append(d)
    a, b = outs
    np.testing.assert_array_equal(np.fromfile(a / "ctr.bin", np.uint64), np.fromfile(b / "ctr.bin", np.uint64))
    names = sorted(n for n in os.listdir(a) if not n.endswith(".bin") or n == "km.bin")
    assert names == sorted(n for n in os.listdir(b) if not n.endswith(".bin") or n == "km.bin")
    for n in names:
        assert (a / n).read_bytes() == (b / n).read_bytes(), n
    if cmd == "stats":
        p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
        _, _, want = O.run(p, reads)
        np.testing.assert_array_equal(np.fromfile(b / "ctr.bin", np.uint64), want)


@pytest.mark.parametrize("cmd", ["stats", "filter", "edit", "filter_stream", "edit_stream"])
def test_cli_threads_under_tsan(tmp_path, cmd):
    """The threaded host pipeline (reader threads, 2 GPU x 2 worker threads,
    writer; hpg-fastq_amd/host/hpgq_pipeline.c) built with ThreadSanitizer
    (`make -C hpg-fastq_amd tsan`; libhpgq itself is not instrumented): no
    race reported, and the outputs equal the plain build's."""
    tsan = os.path.join(os.path.dirname(CLI), "hpg-fastq-tsan")
    if not os.path.exists(tsan):
        pytest.fail("hpg-fastq-tsan not built (make -C hpg-fastq_amd tsan; __graft_entry__.build())")
    reads = O.synth(20000, seed=29, L=150, n_per_1024=6)
    fq = _write(tmp_path, reads)
    outs = []
    cmd, _, mode = cmd.partition("_")
    for exe in (CLI, tsan):
        d = tmp_path / os.path.basename(exe)
        d.mkdir()
        args = [cmd, "-f", fq, "-o", d, "--chunk-mb", 1, "--gpus", 2, "--gpu-workers", 2,
                "--counters-out", d / "ctr.bin", "--quiet", "--read-quality-range", "20,",
                "--read-length-range", "50,"]
        if cmd == "edit":
            args += ["--left-length", 10, "--left-quality-range", "20,"]
        if mode == "stream":
            args += ["--stream-writer"]
        supp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize", "tsan.supp")
        env = dict(os.environ, TSAN_OPTIONS=f"halt_on_error=1:second_deadlock_stack=1:suppressions={supp}")
        # (TSan's shadow layout needs the address-space randomisation off:
        # setarch -R, a fresh process that execs the CLI before any GPU use)
        pre = ["setarch", os.uname().machine, "-R"] if exe == tsan else []
        r = subprocess.run(pre + [exe] + [str(a) for a in args], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
        outs.append(d)
    a, b = outs
    np.testing.assert_array_equal(np.fromfile(a / "ctr.bin", np.uint64), np.fromfile(b / "ctr.bin", np.uint64))
    for n in sorted(os.listdir(a)):
        assert (a / n).read_bytes() == (b / n).read_bytes(), n
