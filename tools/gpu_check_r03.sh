# round 3 check (gpurun): the whole GPU suite, then the driver's default bench
# line (C2 + cpu_baseline + e2e)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03/gpu_suite.log 2>&1 || { echo SUITE_FAILED; grep -E "FAILED|Error|error" gpurun_out/r03/gpu_suite.log | head -20; tail -30 gpurun_out/r03/gpu_suite.log; exit 1; }
tail -1 gpurun_out/r03/gpu_suite.log
timeout -k 10 400 python bench.py > gpurun_out/r03/bench_default.json 2> gpurun_out/r03/bench_default.err || { tail -20 gpurun_out/r03/bench_default.err; exit 2; }
cat gpurun_out/r03/bench_default.json
