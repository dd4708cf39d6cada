#!/bin/bash
# round 4, call V: single-end edit with the next unit's trim lines warmed into
# L2 one group before its prologue (HPGQ_EDIT_WARM 1, the product) against
# no warming (ab/libhpgq_nowarm.so): edit parity tests, C4 / c4_noor A/B and
# FETCH_SIZE for C4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_engine_gpu.py tests/test_fuzz_gpu.py tests/test_fullsize_gpu.py -k "edit or c4 or fuzz" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 3
NW=$PWD/hpg-fastq_amd/ab/libhpgq_nowarm.so
for cfg in c4 c4_noor; do
  for v in warm nowarm warm nowarm warm nowarm; do
    if [ $v = nowarm ]; then L=$NW; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
for v in warm nowarm; do
  if [ $v = nowarm ]; then L=$NW; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch_$v -o run --output-format csv -- python tools/prof_engine.py --mode edit --reads 12500000 --L 150 --iters 3 > $O/fetch_$v.log 2>&1 || exit 6
done
