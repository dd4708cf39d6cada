# CGR fill time per k (occupancy probe): rocprofv3 kernel stats for k in $KS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cgrk
export TMPDIR=/tmp
for k in ${KS:-5 6 7}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cgrk/k$k -o run --output-format csv -- python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 3 --k $k > gpurun_out/cgrk/k$k.log 2>&1 || exit $?
done
