"""The drop-in binding as INTEGRATION.md writes it (tools/dropin_bench.c):
SoA batches of the reference's 10,000 reads (src/stats_options.c:22), packed
into the ctx's staging slot (hpgq_host_batch) or into malloc'd buffers,
packed from AoS reads, hpgq_run_host + hpgq_sync per batch (or, for the stats
worker that needs no mask, one hpgq_sync per worker at the end), one ctx per worker
thread (src/stats_options.c:21: 2 threads) -- the summed counters and every
mask equal the oracle's over the same FASTQ file.  Also the host path's
contract: several hpgq_run_host calls in flight before one hpgq_sync."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

import hpgfastq as H
import oracle_lib as O
from fastq_io import read_fastq

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tools", "dropin_bench")


@pytest.fixture(scope="module")
def fastq(tmp_path_factory):
    d = tmp_path_factory.mktemp("dropin")
    gen = str(d / "fqgen")
    subprocess.run(["gcc", "-O2", "-fopenmp", os.path.join(ROOT, "tools", "fqgen.c"), "-o", gen], check=True)
    path = str(d / "in.fq")
    subprocess.run([gen, path, "123457", "150", "2"], check=True)
    return path


@pytest.mark.parametrize("threads,batch,copy,nosync", [
    (2, 10000, False, False), (1, 997, False, False), (3, 4096, False, False),
    (2, 10000, True, False), (3, 4096, True, False),
    (2, 10000, False, True), (1, 997, False, True), (3, 4096, True, True)])
def test_dropin_worker_matches_oracle(fastq, tmp_path, threads, batch, copy, nosync):
    """copy=False: the worker packs into the ctx's staging slot (hpgq_host_batch);
    copy=True: into malloc'd buffers that hpgq_run_host copies.  nosync: the
    stats worker without a mask or a per-batch hpgq_sync (one sync per worker
    at the end; bench --config dropin's value) -- counters only."""
    assert os.path.exists(HARNESS), "build with make -C hpg-fastq_amd"
    ctr, msk = str(tmp_path / "ctr.bin"), str(tmp_path / "mask.bin")
    out = subprocess.run([HARNESS, fastq, "--batch", str(batch), "--threads", str(threads), "--c2",
                          "--counters", ctr, "--repeat", "2"] + (["--mask", msk] if not nosync else [])
                         + (["--copy"] if copy else []) + (["--no-sync"] if nosync else []),
                         check=True, capture_output=True, text=True, timeout=300)
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["staging"] == ("copy" if copy else "in_place")
    assert rec["sync"] == ("once per worker at the end" if nosync else "per batch")
    reads = read_fastq(fastq)
    assert rec["reads"] == reads.n
    p = H.stats_params(lmax=1024, read_quality_range="20,", read_length_range="50,")
    m_o, _t, c_o = O.run(p, reads)
    if not nosync:
        np.testing.assert_array_equal(np.fromfile(msk, np.uint8), m_o)
    np.testing.assert_array_equal(np.fromfile(ctr, np.uint64), c_o)


@pytest.mark.parametrize("edit", [False, True])
def test_host_path_calls_in_flight(edit):
    """Five hpgq_run_host calls before one hpgq_sync: the two staging slots
    are reused, every batch's mask / trims reach its own arrays, and the
    caller's input buffers are free to change as soon as a call returns."""
    if edit:
        p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                          right_length=30, right_quality_range="20,", max_N=2)
    else:
        p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    batches = [O.synth(n, seed=40 + i, L=150, trunc_pct=10, n_per_1024=8, first=1000 * i)
               for i, n in enumerate([30000, 1, 25000, 7777, 40000])]
    masks = [np.full(b.n, 7, np.uint8) for b in batches]
    trims = [np.zeros(b.n, np.uint32) for b in batches]
    with H.Engine(p) as e:
        for b, m, t in zip(batches, masks, trims):
            seq, qual = b.seq.copy(), b.qual.copy()
            hb = H.engine.host_batch(seq, qual, b.idx)
            e.run_host(hb, None, m, t if edit else None)
            seq[:] = ord("N")   # reused by the caller right away
            qual[:] = 0
        e.sync()
        got = e.counters()
    want = np.zeros_like(got)
    for b, m, t in zip(batches, masks, trims):
        m_o, t_o, c_o = O.run(p, b)
        np.testing.assert_array_equal(m, m_o)
        if edit:
            np.testing.assert_array_equal(t, t_o)
        want += c_o
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("paired,edit", [(False, False), (False, True), (True, False), (True, True)])
def test_host_batch_in_place(paired, edit):
    """hpgq_host_batch + hpgq_run_host (the batch written into the staging slot,
    no host copy), mixed with copied batches on the same ctx and several calls
    in flight: masks, trims and counters equal the oracle's."""
    kw = dict(left_length=10, left_quality_range="20,", right_length=30, right_quality_range="20,")
    p = (H.edit_params(lmax=150, stats=True, **kw) if edit
         else H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,"))
    p.paired = 1 if paired else 0
    mates = 2 if paired else 1
    sizes = [20000, 1, 0, 9999, 30000, 4096]   # (an empty batch in place: reserved, nothing to run)
    bat = [[O.synth(n, seed=70 + i, L=150, trunc_pct=10, n_per_1024=8, first=1000 * i, mate=m)
            for m in range(mates)] for i, n in enumerate(sizes)]
    masks = [np.full(n, 7, np.uint8) for n in sizes]
    trims = [np.zeros(n * mates, np.uint32) for n in sizes]
    with H.Engine(p) as e:
        for i, (bs, m, t) in enumerate(zip(bat, masks, trims)):
            if i % 2 == 0:   # in place
                e.run_host_in_place([(b.seq, b.qual, b.idx) for b in bs], m, t if edit else None)
            else:            # copied
                hbs = [H.engine.host_batch(b.seq, b.qual, b.idx) for b in bs]
                e.run_host(hbs[0], hbs[1] if paired else None, m, t if edit else None)
            if i == 2:
                e.sync()
        e.sync()
        got = e.counters()
    want = np.zeros_like(got)
    for bs, m, t in zip(bat, masks, trims):
        m_o, t_o, c_o = O.run(p, bs[0], bs[1] if paired else None)
        np.testing.assert_array_equal(m, m_o)
        if edit:
            np.testing.assert_array_equal(t, t_o)
        want += c_o
    np.testing.assert_array_equal(got, want)


def test_read_counters_delivers_host_outputs():
    """hpgq_read_counters synchronises the ctx and, like hpgq_sync, hands the
    pending host-path masks / trims to the caller's arrays; a ctx
    closed with outputs pending drops them (never writes them)."""
    p = H.edit_params(lmax=150, stats=True, left_length=10, left_quality_range="20,",
                      right_length=30, right_quality_range="20,", read_quality_range="20,")
    reads = [O.synth(5000, seed=90 + i, L=150, trunc_pct=10, first=7000 * i) for i in range(2)]
    masks = [np.full(r.n, 7, np.uint8) for r in reads]
    trims = [np.zeros(r.n, np.uint32) for r in reads]
    with H.Engine(p) as e:
        for r, m, t in zip(reads, masks, trims):
            e.run_host(H.engine.host_batch(r.seq, r.qual, r.idx), None, m, t)
        got = e.counters()          # no hpgq_sync before it
        for r, m, t in zip(reads, masks, trims):
            m_o, t_o, _ = O.run(p, r)
            np.testing.assert_array_equal(m, m_o)
            np.testing.assert_array_equal(t, t_o)
        want = sum(O.run(p, r)[2] for r in reads)
        np.testing.assert_array_equal(got, want)
        pending = np.full(reads[0].n, 7, np.uint8)
        e.run_host(H.engine.host_batch(reads[0].seq, reads[0].qual, reads[0].idx), None, pending, None)
    assert (pending == 7).all()     # dropped by hpgq_close: untouched
