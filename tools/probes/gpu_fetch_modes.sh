# FETCH_SIZE per prof_engine mode (run via gpurun): MODES="stats nofail c2"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fm
for m in ${MODES:-stats nofail c2}; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/fm/$m -o run --output-format csv -- python tools/prof_engine.py --mode $m --iters 2 ${ARGS} > gpurun_out/fm/$m.log 2>&1 || exit 3
done
