#!/bin/bash
# round 4, call S: bench.py's own launcher with 4 rank processes sharing the
# one GPU (RCCL socket transport between them): C2 and C5 lines with
# n_gpus 4 and rccl_ranks 4 (the 8-GPU xGMI run is the driver's)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 4 --share-device --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/c2_n4.json 2> $O/c2_n4.err || exit 3
timeout -k 10 300 python bench.py --gpus 4 --share-device --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_n4.json 2> $O/c5_n4.err || exit 4
