#!/bin/bash
# round 4, call H: the segmented kernels' stream loads with the nt cache
# policy (ab/libhpgq_nt.so, HPGQ_STREAM_CPOL 2) against the product: edit
# family + C2 bench A/B (alternating) and FETCH_SIZE per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
NT=$PWD/hpg-fastq_amd/ab/libhpgq_nt.so
BASE=$PWD/hpg-fastq_amd/libhpgq.so
for cfg in c4 c4_pe c2 c4_noor; do
  for v in base nt base nt; do
    if [ $v = nt ]; then L=$NT; else L=$BASE; fi
    HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
for spec in c4:edit:12500000 c4_pe:pe_edit:10000000; do
  IFS=: read cfg mode n <<< "$spec"
  for v in base nt; do
    if [ $v = nt ]; then L=$NT; else L=$BASE; fi
    HPGQ_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch_${cfg}_$v -o run --output-format csv -- python tools/prof_engine.py --mode $mode --reads $n --L 150 --iters 3 > $O/fetch_${cfg}_$v.log 2>&1 || exit 5
  done
done
