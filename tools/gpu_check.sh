# tests + short bench + kernel-trace profile on one GPU (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench1.log 2>&1 || exit 3
if [ "${PROFILE:-1}" = "1" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
fi
