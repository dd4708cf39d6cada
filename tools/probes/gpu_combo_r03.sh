set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "adaptive or mixed or lmax1024 or routes or long" > gpurun_out/r03/engine_subset.log 2>&1 || { tail -30 gpurun_out/r03/engine_subset.log; exit 1; }
tail -1 gpurun_out/r03/engine_subset.log
bash tools/probes/gpu_cgrv_split.sh
