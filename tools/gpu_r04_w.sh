#!/bin/bash
# round 4, call W2 (probe): what the edit unit prologue's trim round trip costs.
# Timing-only builds: without trim gathers or trims (ab/libhpgq_notrim1.so),
# and with the trims computed but not applied (ab/libhpgq_notrim2.so); both
# stream the untrimmed reads (MORE bytes); notrim3: trims from made-up windows
# (no gathers), not applied; against the product, C4 and c4_pe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04w2
mkdir -p $O
for cfg in c4 c4_pe; do
  for v in base nt1 nt2 nt3 base nt1 nt2 nt3; do
    if [ $v = base ]; then L=$PWD/hpg-fastq_amd/libhpgq.so; else L=$PWD/hpg-fastq_amd/ab/libhpgq_notrim${v#nt}.so; fi
    HPGQ_LIB_PATH=$L HPGQ_BENCH_NOCHECK=1 timeout -k 10 180 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 4
  done
done
