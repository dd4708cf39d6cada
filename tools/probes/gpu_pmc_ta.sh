# TA/TCP load-path counters for the CGR fill kernel (separate --pmc passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcta
export TMPDIR=/tmp
A="python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 2"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE TA_BUFFER_READ_WAVEFRONTS_sum -d gpurun_out/pmcta/p1 -o run --output-format csv -- $A > gpurun_out/pmcta/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/pmcta/p2 -o run --output-format csv -- $A > gpurun_out/pmcta/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_LATENCY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum -d gpurun_out/pmcta/p3 -o run --output-format csv -- $A > gpurun_out/pmcta/p3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum -d gpurun_out/pmcta/p4 -o run --output-format csv -- $A > gpurun_out/pmcta/p4.log 2>&1
