# occupancy / variant sweep of the C2 bench (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in 4 5 6; do
  HPGQ_TRI_WAVES=$w timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_w$w.log 2>&1 || exit 3
done
