#!/bin/bash
# round 4, call N: edit trim windows loaded dword-aligned (the product) against
# the unaligned 16-byte loads (ab/libhpgq_trua.so): edit parity tests, then
# C4 / c4_pe / c4_noor A/B (alternating) and TA busy + FETCH for C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_engine_gpu.py tests/test_fuzz_gpu.py tests/test_fullsize_gpu.py -k "edit or c4 or fuzz" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
UA=$PWD/hpg-fastq_amd/ab/libhpgq_trua.so
for cfg in c4 c4_pe c4_noor; do
  for v in al ua al ua; do
    if [ $v = ua ]; then L=$UA; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
for v in al ua; do
  if [ $v = ua ]; then L=$UA; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  A="python tools/prof_engine.py --mode edit --reads 12500000 --L 150 --iters 3"
  HPGQ_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $O/ta_$v -o run --output-format csv -- $A > $O/ta_$v.log 2>&1 || exit 5
  HPGQ_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch_$v -o run --output-format csv -- $A > $O/fetch_$v.log 2>&1 || exit 6
done
