set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmccgr
export TMPDIR=/tmp
A="python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR -d gpurun_out/pmccgr/p1 -o run --output-format csv -- $A > gpurun_out/pmccgr/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d gpurun_out/pmccgr/p2 -o run --output-format csv -- $A > gpurun_out/pmccgr/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/pmccgr/p3 -o run --output-format csv -- $A > gpurun_out/pmccgr/p3.log 2>&1
