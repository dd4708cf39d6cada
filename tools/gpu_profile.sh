# Round profiles (gpurun): the driver's bench command under the kernel trace
# (with --no-e2e: the e2e leg's CLI processes launch the same kernel names on
# 256 MB chunks and would enter the trace), then per config a short bench line
# and the HBM PMC passes (FETCH_SIZE / WRITE_SIZE, one per run) on the same
# kernels and batch, the SQ passes for C2 and the LDS passes for C5.
#   P=gpurun_out/prof5 SPECS="cfg:mode:reads:L[:extra] ..." bash tools/gpu_profile.sh
# Then: python tools/profile_report.py --round r05 --prof gpurun_out/prof5
# (which also writes this session's PMC bytes into the committed bench lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${P:-gpurun_out/prof}
mkdir -p $P
if [ -z "$SKIP_TRACE" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-e2e > $P/bench.json 2> $P/trace.err || exit 3
fi
for spec in ${SPECS:-c2:c2:10000000:150 c3:pe:10000000:150 c4:edit:12500000:150 c4_noor:edit_noor:12500000:150 c4_pe:pe_edit:10000000:150 c5:cgr:5000000:250 c5_valid:cgrv:5000000:250 c2_lr:lr:10000000:150 c2_250:c2:5000000:250 c2_kmers:c2:10000000:150:--kmers}; do
  IFS=: read cfg mode n L extra <<< "$spec"
  A="python tools/prof_engine.py --mode $mode --reads $n --L $L --iters 3 $extra"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/btrace_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $P/bench_$cfg.json 2> $P/bench_$cfg.err || exit 4
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/fetch_$cfg -o run --output-format csv -- $A > $P/fetch_$cfg.log 2>&1 || exit 5
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/write_$cfg -o run --output-format csv -- $A > $P/write_$cfg.log 2>&1 || exit 6
done
A="python tools/prof_engine.py --mode c2 --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d $P/sq1 -o run --output-format csv -- $A > $P/sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $P/sq2 -o run --output-format csv -- $A > $P/sq2.log 2>&1 || exit 7
for mode in cgr cgrv; do
  A="python tools/prof_engine.py --mode $mode --reads 5000000 --L 250 --iters 3"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d $P/lds1_$mode -o run --output-format csv -- $A > $P/lds1_$mode.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $P/lds2_$mode -o run --output-format csv -- $A > $P/lds2_$mode.log 2>&1 || exit 8
done
A="python tools/prof_engine.py --mode c2 --kmers --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $P/lds2_kmers -o run --output-format csv -- $A > $P/lds2_kmers.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $P/ta_kmers -o run --output-format csv -- $A > $P/ta_kmers.log 2>&1 || exit 9
