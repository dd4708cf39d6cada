# engine kernel counters per mode (gpurun): kernel trace, instruction mix,
# wait cycles, HBM bytes (FETCH_SIZE / WRITE_SIZE in their own passes).
#   MODES="pe pe_edit" bash tools/gpu_pmc_engine_r03.sh; python tools/pmc_report.py gpurun_out/pmceng_<mode> engine_tri
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mode in ${MODES:-pe pe_edit}; do
  D=gpurun_out/pmceng_$mode
  mkdir -p $D
  A="python tools/prof_engine.py --mode $mode --reads ${READS:-10000000} --iters 2"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $A > $D/trace.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d $D/p1 -o run --output-format csv -- $A > $D/p1.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d $D/p2 -o run --output-format csv -- $A > $D/p2.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $A > $D/fetch.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- $A > $D/write.log 2>&1 || exit 3
done
