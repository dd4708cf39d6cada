#!/bin/bash
# round 4: call C (pipeline trace, spill-fix A/B, drop-in) + the k-mer kernel call
bash tools/gpu_r04_kmers.sh || exit $?
bash tools/gpu_r04_c.sh || exit $?
