# round 3: CGR valid-reads path: tests, then kernel time by share of skipped reads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py > gpurun_out/r03/cgr_tests.log 2>&1 || { tail -30 gpurun_out/r03/cgr_tests.log; exit 1; }
tail -1 gpurun_out/r03/cgr_tests.log
bash tools/probes/gpu_cgrv_split.sh
