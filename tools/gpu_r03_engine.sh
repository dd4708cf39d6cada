# round 3: segmented edit variants (edit + N / out-of-range, paired-end edit),
# the host path (staging slots, drop-in harness) and the new bench configs (gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 900 $T ${TESTS:-tests/test_engine_gpu.py tests/test_fuzz_gpu.py tests/test_dropin_gpu.py} > gpurun_out/r03/engine_tests.log 2>&1 || { echo ENGINE_TESTS_FAILED; tail -40 gpurun_out/r03/engine_tests.log; exit 1; }
tail -2 gpurun_out/r03/engine_tests.log
for c in ${CFGS:-c4 c4_noor c4_pe c5 c5_valid}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/bench_$c.json 2> gpurun_out/r03/bench_$c.err || { echo BENCH_FAILED $c; tail -5 gpurun_out/r03/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r03/bench_$c.json')); r=d['roofline']; print('$c', d['value'], d['unit'], r['avg_launch_us'], r['frac'], r['kernel'])"
done
if [ -z "$NO_DROPIN" ]; then
  gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen && timeout -k 10 120 /tmp/fqgen /dev/shm/dropin.fq 4000000 150 2 || exit 4
  for t in 1 2 4; do
    timeout -k 10 300 tools/dropin_bench /dev/shm/dropin.fq --threads $t --batch 10000 --c2 --repeat 3 | tee -a gpurun_out/r03/dropin.log || { rm -f /dev/shm/dropin.fq; exit 5; }
  done
  rm -f /dev/shm/dropin.fq
fi
