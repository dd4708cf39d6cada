# C2/C3/C4 bench per libhpgq variant and occupancy (run via gpurun):
# RUNS="main:5 s3:4 ..." (variant:HPGQ_TRI_WAVES; "main" = the tree's build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for spec in ${RUNS:-main:5}; do
  IFS=: read v w <<< "$spec"
  if [ "$v" = main ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so; fi
  export HPGQ_TRI_WAVES=$w
  if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/var/test_${v}_$w.log 2>&1 || exit 3
  fi
  for c in ${CFGS:-c2}; do
    timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var/bench_${v}_${w}_$c.json 2> gpurun_out/var/bench_${v}_${w}_$c.err || exit 4
  done
done
