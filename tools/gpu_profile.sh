# Round profile (run via gpurun): tests, full bench line, rocprofv3 kernel-trace
# stats of the bench itself, and per config (c2..c5) a short bench line plus the
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate passes, kernel trace only)
# on the same kernels and batch size.
# Then: python tools/profile_report.py --round rNN   (here, on the merged output)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/prof/pytest_gpu.log 2>&1 || exit 3
fi
# the driver's exact bench command under the kernel trace: its JSON line and
# the trace's per-kernel averages come from the same run
[ -n "$SKIP_BENCH" ] || timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof/bench.json 2> gpurun_out/prof/trace.err || exit 3
for spec in ${CFGS:-c2:c2:10000000:150 c3:pe:10000000:150 c4:edit:12500000:150 c5:cgr:5000000:250 c2_lr:lr:10000000:150 c2_250:c2:5000000:250}; do
  IFS=: read cfg mode n L <<< "$spec"
  A="python tools/prof_engine.py --mode $mode --reads $n --L $L --iters 3"
  timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_$cfg.json 2> gpurun_out/prof/bench_$cfg.err || exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/prof/fetch_$cfg -o run --output-format csv -- $A > gpurun_out/prof/fetch_$cfg.log 2>&1 || exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/prof/write_$cfg -o run --output-format csv -- $A > gpurun_out/prof/write_$cfg.log 2>&1 || exit 3
done
[ -n "$SKIP_BENCH" ] || timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d gpurun_out/prof/sq1 -o run --output-format csv -- python tools/prof_engine.py --mode c2 --iters 3 > gpurun_out/prof/sq1.log 2>&1 || exit 3
[ -n "$SKIP_BENCH" ] || timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d gpurun_out/prof/sq2 -o run --output-format csv -- python tools/prof_engine.py --mode c2 --iters 3 > gpurun_out/prof/sq2.log 2>&1
