# PMC passes for the engine kernel (separate passes; kernel-trace only, no sys/runtime trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
MODE=${MODE:-c2}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 -d gpurun_out/pmc/$1 -o run --output-format csv -- python tools/prof_engine.py --mode $MODE --iters 3 > gpurun_out/pmc/$1.log 2>&1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/trace -o run --output-format csv -- python tools/prof_engine.py --mode $MODE --iters 5 > gpurun_out/pmc/trace.log 2>&1 &&
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" &&
run p2 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" &&
run p3 "FETCH_SIZE" &&
run p4 "WRITE_SIZE" &&
run p5 "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
