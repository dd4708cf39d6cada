# engine A/B (run via gpurun): VARIANTS="main prio1 ..." x CFGS="c2 c4" bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/engab
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so; fi
  for c in ${CFGS:-c2}; do
    timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/engab/${v}_$c.json 2> gpurun_out/engab/${v}_$c.err || exit 4
  done
done
