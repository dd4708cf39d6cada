# probe: C5 stream kernel with / without the start-bit LDS read in the tile loop (timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5noso
export TMPDIR=/tmp
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 6 --mode cgr"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5noso/base -o run --output-format csv -- $A > gpurun_out/c5noso/base.log 2>&1 || exit 1
HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/noso/libhpgq.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5noso/noso -o run --output-format csv -- $A > gpurun_out/c5noso/noso.log 2>&1 || exit 2
