# probe: CGR stream kernel cost by share of skipped reads (ONLY_VALID_READS), 5 M x 250 bp
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cgrv
export TMPDIR=/tmp
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 5"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cgrv/all -o run --output-format csv -- $A --mode cgr > gpurun_out/cgrv/all.log 2>&1 || exit 1
for P in 0 1 5 20; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cgrv/p$P -o run --output-format csv -- $A --mode cgrv --invalid-pct $P > gpurun_out/cgrv/p$P.log 2>&1 || exit 2
done
