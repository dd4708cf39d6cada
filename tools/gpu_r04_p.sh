#!/bin/bash
# round 4, call P: the CGR stream kernel's idx window kept raw until use (no
# wait at the loop merge for the prefetched tiles; the product, depth 3) against
# the select at the merge (ab/libhpgq_rw0.so) and raw window at depth 2
# (ab/libhpgq_rwd2.so): CGR parity tests, C5 / c5_valid A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
for cfg in c5 c5_valid; do
  for v in raw rw0 rwd2 raw rw0 rwd2; do
    if [ $v = raw ]; then L=$PWD/hpg-fastq_amd/libhpgq.so; else L=$PWD/hpg-fastq_amd/ab/libhpgq_$v.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
