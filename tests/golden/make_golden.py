"""Regenerate the committed synthetic vectors tests/golden/synth_*.npz.

Inputs: the counter-based synthetic generator (oracle_synth, same as bench.py
and the GPU tests).  Expected outputs: the pure-Python restatement
oracle/pyref.py (plain loops over the reference's rules, independent of the C
oracle and of the HIP engine).  tests/test_oracle_cpu.py checks that the C
oracle reproduces them; tests/test_engine_gpu.py that the GPU does.

  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "hpg-fastq_amd"), ROOT, os.path.join(ROOT, "tests")]

import hpgfastq as H  # noqa: E402
import oracle_lib as O  # noqa: E402
from oracle import pyref  # noqa: E402


def save(name, p, r1, r2=None, **extra):
    pr = pyref.default_params(**p.as_dict())
    mask, trims, ctr = pyref.run(pr, r1.pairs(), r2.pairs() if r2 is not None else None)
    d = dict(params=json.dumps(p.as_dict()), seq=r1.seq, qual=r1.qual, idx=r1.idx,
             mask=np.array(mask, np.uint8), trim=np.array(trims, np.uint32),
             counters=np.array(ctr, np.uint64))
    if r2 is not None:
        d.update(seq2=r2.seq, qual2=r2.qual, idx2=r2.idx)
    d.update(extra)
    np.savez_compressed(os.path.join(HERE, name), **d)
    print(name, r1.n, "reads")


def main():
    # C2: stats + filter, 150 bp (BASELINE configs[1] flags)
    r = O.synth(400, seed=2, L=150)
    save("synth_c2_filter.npz", H.stats_params(lmax=150, read_quality_range="20,",
                                               read_length_range="50,"), r)
    # C4: edit + stats
    r = O.synth(300, seed=4, L=150)
    save("synth_c4_edit.npz", H.edit_params(lmax=150, stats=True, left_length=10,
                                            left_quality_range="20,", right_length=30,
                                            right_quality_range="20,"), r)
    # C3: paired-end, pair passes iff both mates pass
    r1 = O.synth(200, seed=3, L=150, mate=0)
    r2 = O.synth(200, seed=3, L=150, mate=1)
    pp = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    pp.paired = 1
    save("synth_c3_pe.npz", pp, r1, r2)
    # every filter knob, 250 bp, phred33
    r = O.synth(300, seed=6, L=250, trunc_pct=20, n_per_1024=20)
    save("synth_filter_all_250.npz",
         H.stats_params(lmax=250, read_quality_range="18,38", read_length_range="40,240",
                        max_N=3, max_out_of_quality=30, left_length=12, left_quality_range="22,",
                        right_length=20, right_quality_range="10,"), r)
    # C5: chaos game k=7, 250 bp + homopolymer reads (the carried-state case)
    r = O.synth(60, seed=5, L=250)
    pairs = r.pairs() + [(b"A" * 250, b"I" * 250), (b"T" * 120, b"5" * 120),
                         (b"ACGT" * 20 + b"A" * 60, b"?" * 140)]
    rc = O.Reads.from_pairs(pairs)
    ts, tq, wc = pyref.cgr_fill(7, 33, rc.pairs())
    np.savez_compressed(os.path.join(HERE, "synth_cgr_k7.npz"),
                        params=json.dumps(H.params_default(lmax=250).as_dict()),
                        seq=rc.seq, qual=rc.qual, idx=rc.idx, k=np.int32(7),
                        table_seq=np.array(ts, np.uint32), table_q=np.array(tq, np.uint32),
                        word_count=np.uint32(wc))
    print("synth_cgr_k7.npz", rc.n, "reads")


if __name__ == "__main__":
    main()
