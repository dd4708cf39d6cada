# round 3: --kmers (id-major conflict-free table, two lanes per read) and the host path:
# tests, c2_kmers / dropin bench lines, kmers trace + HBM bytes + SQ/LDS counters (gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03 gpurun_out/pmckm2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmers_gpu.py tests/test_dropin_gpu.py > gpurun_out/r03/kmers_tests.log 2>&1 || { tail -30 gpurun_out/r03/kmers_tests.log; exit 1; }
tail -1 gpurun_out/r03/kmers_tests.log
timeout -k 10 300 python bench.py --config c2_kmers --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/bench_c2_kmers.json 2> gpurun_out/r03/bench_c2_kmers.err || { tail -5 gpurun_out/r03/bench_c2_kmers.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/r03/bench_c2_kmers.json')); r=d['roofline']; print('c2_kmers', d['value'], r['avg_launch_us'], r['frac'])"
timeout -k 10 300 python bench.py --config dropin --steps 5 > gpurun_out/r03/bench_dropin.json 2> gpurun_out/r03/bench_dropin.err || { tail -5 gpurun_out/r03/bench_dropin.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/r03/bench_dropin.json')); print('dropin', d['value'], d['harness']['mreads_s_mean'])"
A="python tools/prof_engine.py --mode c2 --kmers --iters 2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmckm2/trace -o run --output-format csv -- $A > gpurun_out/pmckm2/trace.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmckm2/fetch -o run --output-format csv -- $A > gpurun_out/pmckm2/fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmckm2/write -o run --output-format csv -- $A > gpurun_out/pmckm2/write.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d gpurun_out/pmckm2/p1 -o run --output-format csv -- $A > gpurun_out/pmckm2/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/pmckm2/p3 -o run --output-format csv -- $A > gpurun_out/pmckm2/p3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d gpurun_out/pmckm2/ta -o run --output-format csv -- $A > gpurun_out/pmckm2/ta.log 2>&1
