# CGR stream kernel counters (all reads / ONLY_VALID_READS), one pass per
# counter group (gpurun): instruction mix, wait cycles, LDS bank conflicts,
# HBM bytes.  Summaries: python tools/pmc_report.py gpurun_out/pmccgr_<mode> cgr_stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mode in ${MODES:-cgr cgrv}; do
  D=gpurun_out/pmccgr_$mode
  mkdir -p $D
  A="python tools/prof_engine.py --mode $mode --reads 5000000 --L 250 --iters 2"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $A > $D/trace.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d $D/p1 -o run --output-format csv -- $A > $D/p1.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d $D/p2 -o run --output-format csv -- $A > $D/p2.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $D/p3 -o run --output-format csv -- $A > $D/p3.log 2>&1 &&
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- $A > $D/fetch.log 2>&1 || exit 3
done
