# probe: C5 with register-only start bits: CGR tests, then timing vs the LDS-bitmap build (ab/noso: no read
# back, timing only) and kernel time by share of skipped reads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5g gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py > gpurun_out/r03/cgr_tests.log 2>&1 || { tail -30 gpurun_out/r03/cgr_tests.log; exit 1; }
tail -1 gpurun_out/r03/cgr_tests.log
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 6"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5g/new -o run --output-format csv -- $A --mode cgr > gpurun_out/c5g/new.log 2>&1 || exit 2
HPGQ_LIB_PATH=$PWD/hpg-fastq_amd/ab/noso/libhpgq.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5g/noso -o run --output-format csv -- $A --mode cgr > gpurun_out/c5g/noso.log 2>&1 || exit 3
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5g/newv -o run --output-format csv -- $A --mode cgrv > gpurun_out/c5g/newv.log 2>&1 || exit 4
for C in c5 c5_valid; do
  timeout -k 10 300 python bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5g/bench_$C.json 2> gpurun_out/c5g/bench_$C.err || { tail -5 gpurun_out/c5g/bench_$C.err; exit 5; }
  python -c "import json; d=json.load(open('gpurun_out/c5g/bench_$C.json')); r=d['roofline']; print('$C', d['value'], r['avg_launch_us'], r['frac'])"
done
