#!/bin/bash
# round 4, call O: the committed c2_kmers profile with the aligned windows
# (tools/gpu_profile_r04.sh, c2_kmers only, no driver trace), then the full
# GPU suite once more
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SKIP_TRACE=1 SPECS="c2_kmers:c2:10000000:150:--kmers" bash tools/gpu_profile_r04.sh || exit $?
mkdir -p gpurun_out/r04o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o/gpu_suite.log 2>&1 || exit 3
