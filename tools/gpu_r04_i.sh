#!/bin/bash
# round 4, call I: the committed profiles (tools/gpu_profile_r04.sh) and the
# tmpfs fill probe (the stored-output bound of the mapped writer)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04i
gcc -O2 -pthread tools/ubench/tmpfs_fill.c -o /tmp/tmpfs_fill || exit 2
timeout -k 10 120 /tmp/tmpfs_fill /dev/shm 3000000000 > gpurun_out/r04i/tmpfs_fill.jsonl 2>&1 || exit 3
bash tools/gpu_profile_r04.sh || exit $?
