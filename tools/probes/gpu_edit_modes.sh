# edit-kernel decomposition (run via gpurun): kernel-trace averages per prof_engine mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/em
for m in ${MODES:-c2 edit edit0 editL editR}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/em/$m -o run --output-format csv -- python tools/prof_engine.py --mode $m --reads 12500000 --iters 5 > gpurun_out/em/$m.log 2>&1 || exit 3
done
