set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py > gpurun_out/r03/cgr_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/cgr_tests.log; exit 1; }
tail -3 gpurun_out/r03/cgr_tests.log
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/c5.json 2>gpurun_out/r03/c5.err && cat gpurun_out/r03/c5.json
timeout -k 10 300 python bench.py --config c5_valid --steps 10 --warmup 3 > gpurun_out/r03/c5v.json 2>gpurun_out/r03/c5v.err && cat gpurun_out/r03/c5v.json
