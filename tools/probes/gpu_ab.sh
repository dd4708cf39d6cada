# A/B of two libhpgq builds on one box: alternate runs of one config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
C=${CFG:-c2}
for i in 1 2; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > gpurun_out/ab/new_$i.json 2>/dev/null || exit 3
  HPGQ_LIB_PATH=$PWD/${OLD:-hpg-fastq_amd/ab/libhpgq_2afbe5b.so} timeout -k 10 300 python bench.py --config $C --no-cpu-baseline > gpurun_out/ab/old_$i.json 2>/dev/null || exit 4
done
