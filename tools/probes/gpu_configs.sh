# all bench configs (run via gpurun); each step time-limited, stop at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/cfg/pytest_gpu.log 2>&1 || exit 3
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  timeout -k 10 600 python bench.py --config $c > gpurun_out/cfg/bench_$c.json 2> gpurun_out/cfg/bench_$c.err || exit 4
done
