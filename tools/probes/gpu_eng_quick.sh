set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/eng
timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng/test.log 2>&1 || exit 3
for c in c2 c4 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/eng/bench_$c.json 2> gpurun_out/eng/bench_$c.err || exit 4
done
