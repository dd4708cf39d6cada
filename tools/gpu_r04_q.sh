#!/bin/bash
# round 4, call Q: --kmers with a two-group window pipeline, two alternating register sets (the product)
# against the one-group pipeline (ab/libhpgq_km1.so): parity tests, c2_kmers
# A/B (alternating) and TA busy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04q2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kmers_gpu.py tests/test_cli_gpu.py -k "kmers" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
for v in d2 d1 d2 d1 d2 d1; do
  if [ $v = d1 ]; then L=$PWD/hpg-fastq_amd/ab/libhpgq_km1.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 240 python bench.py --config c2_kmers --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_$v.jsonl 2>> $O/bench.err || exit 4
done
A="python tools/prof_engine.py --mode c2 --kmers --iters 3"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $O/ta -o run --output-format csv -- $A > $O/ta.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq -o run --output-format csv -- $A > $O/sq.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $A > $O/fetch.log 2>&1 || exit 8
