"""Debug: which reads differ between the engine and the oracle (prints lengths)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hpg-fastq_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import hpgfastq as H  # noqa: E402
import oracle_lib as O  # noqa: E402

reads = O.synth(3000, seed=7, L=300, trunc_pct=30, n_per_1024=20)
p = H.stats_params(lmax=512, read_quality_range="15,", read_length_range="30,")
with H.Engine(p) as e:
    print(e.kernel_chain)
    mask, _ = e.process(reads.seq, reads.qual, reads.idx)
    c = e.counters()
m_o, _, c_o = O.run(p, reads)
lens = np.diff(reads.idx)
bad = np.nonzero(mask != m_o)[0]
print("bad", bad, "len", lens[bad], "gpu", mask[bad], "oracle", m_o[bad])
print("units of 48:", bad // 48, "pos", bad % 48)
for u in sorted(set(bad // 48)):
    ls = lens[u * 48:(u + 1) * 48]
    print(u, "lens", list(ls))
d = np.nonzero(c != c_o)[0]
print("counter diffs", d[:20], c[d[:20]], c_o[d[:20]])
print("deferred to wide:", int(((lens > 156) & (lens <= 252)).sum()), "to catch-all:", int((lens > 252).sum()))
