# round 3: CGR stream pass (all reads / ONLY_VALID_READS): tests, bench lines,
# and the instruction-mix pass of both kernels (gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py > gpurun_out/r03/cgr_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03/cgr_tests.log; exit 1; }
tail -1 gpurun_out/r03/cgr_tests.log
for c in c5 c5_valid; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/bench_$c.json 2> gpurun_out/r03/bench_$c.err || exit 2
  python -c "import json; d=json.load(open('gpurun_out/r03/bench_$c.json')); r=d['roofline']; print('$c', d['value'], r['avg_launch_us'], r['frac'])"
done
for mode in cgr cgrv; do
  D=gpurun_out/pmccgr_$mode
  mkdir -p $D
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d $D/p1 -o run --output-format csv -- python tools/prof_engine.py --mode $mode --reads 5000000 --L 250 --iters 2 > $D/p1.log 2>&1 || exit 3
done
