# round 3: the GPU suite, then bench lines of the engine configs (no CPU / e2e legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/q/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/q/tests.log | head -30; tail -30 gpurun_out/q/tests.log; exit 1; }
  tail -1 gpurun_out/q/tests.log
fi
for c in ${CFGS:-c2 c3 c4}; do
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/q/bench_$c.json 2> gpurun_out/q/bench_$c.err || { tail -20 gpurun_out/q/bench_$c.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/q/bench_$c.json')); r=d['roofline']; print('$c', round(d['value'],1), d['ms_per_step'], r['avg_launch_us'], r['frac'])"
done
