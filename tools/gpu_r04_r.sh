#!/bin/bash
# round 4, call R (final): the c2_kmers profile of the final kernel, the full
# GPU suite, smoke() and the driver's default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SKIP_TRACE=1 SPECS="c2_kmers:c2:10000000:150:--kmers" bash tools/gpu_profile_r04.sh || exit $?
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 5
