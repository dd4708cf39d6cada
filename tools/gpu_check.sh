# GPU suite + bench lines (run via gpurun); output under gpurun_out/check
#   CFGS="c2 c2_1024 ..." selects the extra bench configs (short runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/check
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/check/pytest_gpu.log 2>&1 || exit 3
fi
timeout -k 10 300 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || exit 4
for c in ${CFGS}; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/check/bench_$c.json 2> gpurun_out/check/bench_$c.err || exit 5
done
