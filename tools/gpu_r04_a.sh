#!/bin/bash
# round 4, first GPU call: routing via hpgq_debug_set_route, bench line, then
# the two-rank RCCL tests (ranks share the box's one GPU; socket transport)
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 --timeout-method thread > $O/engine.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-e2e > $O/bench.json 2> $O/bench.err || exit 4
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 200 --timeout-method thread > $O/multirank.log 2>&1 || exit 5
