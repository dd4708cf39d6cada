# C5 bench per libhpgq variant (run via gpurun): VARIANTS="l16p1 l16p0 ..." ("main" = the tree's build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so; fi
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/var/test_$v.log 2>&1 || exit 3
  fi
  timeout -k 10 300 python bench.py --config ${CFG:-c5} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var/bench_$v.json 2> gpurun_out/var/bench_$v.err || exit 4
done
