# Round-2 profiles (run via gpurun): rocprofv3 kernel trace + stats of the exact
# driver bench command (its JSON line is kept beside the trace), and of other
# configs; output under gpurun_out/prof2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/c2 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof2/bench_c2_traced.json 2> gpurun_out/prof2/c2.err || exit 3
for c in ${CFGS}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof2/bench_${c}_traced.json 2> gpurun_out/prof2/$c.err || exit 4
done
