# A/B with traffic (run via gpurun): VARIANTS x CFGS bench lines, then FETCH_SIZE
# per variant for one prof_engine MODE
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/engab
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so; fi
  for c in ${CFGS:-c2}; do
    timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/engab/${v}_$c.json 2> gpurun_out/engab/${v}_$c.err || exit 4
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/engab/fetch_$v -o run --output-format csv -- python tools/prof_engine.py --mode ${MODE:-c2} --iters 2 ${ARGS} > gpurun_out/engab/fetch_$v.log 2>&1 || exit 5
done
