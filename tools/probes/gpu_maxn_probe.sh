# max_N / max_out_of_quality: the segmented filter variant vs the one-read kernel (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/maxn
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/maxn/seg -o run --output-format csv -- python tools/prof_engine.py --mode maxn --iters 5 > gpurun_out/maxn/seg.log 2>&1 || exit 3
HPGQ_KERNEL=single timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/maxn/single -o run --output-format csv -- python tools/prof_engine.py --mode maxn --iters 5 > gpurun_out/maxn/single.log 2>&1 || exit 3
