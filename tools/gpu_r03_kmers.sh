# round 3: --kmers kernel: tests, the c2_kmers bench line, trace + HBM bytes (gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03 gpurun_out/pmckm
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmers_gpu.py > gpurun_out/r03/kmers_tests.log 2>&1 || { tail -30 gpurun_out/r03/kmers_tests.log; exit 1; }
tail -1 gpurun_out/r03/kmers_tests.log
timeout -k 10 300 python bench.py --config c2_kmers --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03/bench_c2_kmers.json 2> gpurun_out/r03/bench_c2_kmers.err || { tail -5 gpurun_out/r03/bench_c2_kmers.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/r03/bench_c2_kmers.json')); r=d['roofline']; print('c2_kmers', d['value'], r['avg_launch_us'], r['frac'])"
A="python tools/prof_engine.py --mode c2 --kmers --iters 2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmckm/trace -o run --output-format csv -- $A > gpurun_out/pmckm/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmckm/fetch -o run --output-format csv -- $A > gpurun_out/pmckm/fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d gpurun_out/pmckm/p1 -o run --output-format csv -- $A > gpurun_out/pmckm/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/pmckm/p3 -o run --output-format csv -- $A > gpurun_out/pmckm/p3.log 2>&1
