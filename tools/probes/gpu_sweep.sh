# variant sweep of the C2 bench (run via gpurun): HPGQ_TRI_WAVES x HPGQ_TRI_UNALIGNED
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
for v in ${SWEEP:-5:0 6:0 5:1 6:1}; do
  w=${v%%:*}; u=${v##*:}
  HPGQ_TRI_WAVES=$w HPGQ_TRI_UNALIGNED=$u timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${w}_${u}.log 2>&1 || exit 3
done
