# probe: C5 stream kernel with every tile load hitting one L2-resident 16 KB region (timing only) vs the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5l2
export TMPDIR=/tmp
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 8 --mode cgr"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5l2/tree -o run --output-format csv -- $A > gpurun_out/c5l2/tree.log 2>&1 || exit 1
HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/l2hot/libhpgq.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5l2/l2hot -o run --output-format csv -- $A > gpurun_out/c5l2/l2hot.log 2>&1 || exit 2
