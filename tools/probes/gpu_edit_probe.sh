# C4 timing probes (run via gpurun): the edit kernel with both trims, none,
# left only, right only, and C2, each under a kernel trace; per-kernel stats
# land in gpurun_out/editp/<mode>/
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/editp
export TMPDIR=/tmp
for m in ${MODES:-c2 edit edit0 editL editR}; do
  n=12500000; [ $m = c2 ] && n=10000000
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/editp/$m -o run --output-format csv -- python tools/prof_engine.py --mode $m --reads $n --iters 5 > gpurun_out/editp/$m.log 2>&1 || exit 3
done
