# CGR fill-kernel time per libhpgq variant (tools/build_ab.sh): VARIANTS="base nolds ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cgrab
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cgrab/$v -o run --output-format csv -- python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 3 --k ${K:-7} > gpurun_out/cgrab/$v.log 2>&1 || exit $?
done
