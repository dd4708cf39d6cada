# full GPU tests, then given configs at given occupancies (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/cfg/pytest_gpu.log 2>&1 || exit 3
for v in ${SWEEP:-c2:5 c3:4}; do
  c=${v%%:*}; w=${v##*:}
  HPGQ_TRI_WAVES=$w timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/sw_${c}_${w}.json 2> gpurun_out/cfg/sw_${c}_${w}.err || exit 4
done
