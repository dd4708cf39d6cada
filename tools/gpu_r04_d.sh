#!/bin/bash
# round 4, call D: --kmers with coalesced meta loads (parity + A/B against
# round 3's kernel ab/libhpgq_km32.so + TA counters), then the C5 ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmers_gpu.py tests/test_cli_gpu.py -k "kmers" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
for v in new km32 new km32 new km32; do
  if [ $v = km32 ]; then L=$PWD/hpg-fastq_amd/ab/libhpgq_km32.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 240 python bench.py --config c2_kmers --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_$v.jsonl 2>> $O/bench.err || exit 4
done
A="python tools/prof_engine.py --mode c2 --kmers --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $O/ta -o run --output-format csv -- $A > $O/ta.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $O/lds -o run --output-format csv -- $A > $O/lds.log 2>&1 || exit 8
bash tools/gpu_c5_ablation_r04.sh || exit $?
