#!/bin/bash
# round 4, call U (probe): what the edit unit prologue's trim round trip costs.
# Timing-only build without trim gathers or trims (ab/libhpgq_notrim.so: it
# streams the untrimmed reads, MORE bytes) against the product, C4 and c4_pe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
for cfg in c4 c4_pe; do
  for v in base nt base nt; do
    if [ $v = nt ]; then L=$PWD/hpg-fastq_amd/ab/libhpgq_notrim.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
    HPGQ_LIB_PATH=$L HPGQ_BENCH_NOCHECK=1 timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
