# SQ counters of the C2 engine kernel (run via gpurun): MODE=c2|edit|pe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
A="python tools/prof_engine.py --mode ${MODE:-c2} --iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d gpurun_out/pmc2/p1 -o run --output-format csv -- $A > gpurun_out/pmc2/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d gpurun_out/pmc2/p2 -o run --output-format csv -- $A > gpurun_out/pmc2/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/pmc2/p3 -o run --output-format csv -- $A > gpurun_out/pmc2/p3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum -d gpurun_out/pmc2/p4 -o run --output-format csv -- $A > gpurun_out/pmc2/p4.log 2>&1
