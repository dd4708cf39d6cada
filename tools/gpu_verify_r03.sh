# round 3 final check: the whole GPU suite, then the driver's default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/v/gpu_suite.log 2>&1 || { echo SUITE_FAILED; grep -E "FAILED|Error" gpurun_out/v/gpu_suite.log | head -20; tail -30 gpurun_out/v/gpu_suite.log; exit 1; }
tail -1 gpurun_out/v/gpu_suite.log
timeout -k 10 600 python bench.py > gpurun_out/v/bench_default.json 2> gpurun_out/v/bench_default.err || { tail -20 gpurun_out/v/bench_default.err; exit 2; }
cat gpurun_out/v/bench_default.json
