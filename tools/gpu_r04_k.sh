#!/bin/bash
# round 4, call K: /dev/shm capacity on the box and which writer the bench's
# e2e filter / edit legs ran (20 M reads, 6.2 GB in)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
df -B1 /dev/shm > $O/df.txt 2>&1
free -b >> $O/df.txt 2>&1
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 5
