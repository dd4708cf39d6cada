set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 600 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || exit 4
