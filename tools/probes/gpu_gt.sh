# round 3: single-end edit trims by phase (GT) -- edit parity tests, then C4 / c4_noor bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "edit or mixed or kat" > gpurun_out/gt/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gt/tests.log | head -30; tail -40 gpurun_out/gt/tests.log; exit 1; }
tail -2 gpurun_out/gt/tests.log
for c in c4 c4_noor; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gt/bench_$c.json 2> gpurun_out/gt/bench_$c.err || { tail -20 gpurun_out/gt/bench_$c.err; exit 2; }
  python -c "import json,sys; d=json.load(open('gpurun_out/gt/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline'])"
done
