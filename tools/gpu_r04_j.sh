#!/bin/bash
# round 4, call J: the full GPU suite, smoke(), and the driver's default bench
# line (with its e2e legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 5
