# probe: CGR stream kernel stall counters (all reads and 5 % skipped) + c5 / c5_valid bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5stall gpurun_out/r03
export TMPDIR=/tmp
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 2"
for M in cgr cgrv; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES -d gpurun_out/c5stall/a_$M -o run --output-format csv -- $A --mode $M > gpurun_out/c5stall/a_$M.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD -d gpurun_out/c5stall/b_$M -o run --output-format csv -- $A --mode $M > gpurun_out/c5stall/b_$M.log 2>&1 || exit 2
done
for C in c5 c5_valid; do
  timeout -k 10 300 python bench.py --config $C --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/bench_$C.json 2> gpurun_out/r03/bench_$C.err || { tail -5 gpurun_out/r03/bench_$C.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/r03/bench_$C.json')); r=d['roofline']; print('$C', d['value'], r['avg_launch_us'], r['frac'])"
done
