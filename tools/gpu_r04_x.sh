#!/bin/bash
# round 4, call X (probe): paired-end edit with each mate's trims fetched and
# finished in turn (HPGQ_PE_TRIM_OVERLAP 0, ab/libhpgq_peov0.so) against both
# mates' trim loads in flight together (the product), c4_pe A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
for v in base ov0 base ov0 base ov0; do
  if [ $v = base ]; then L=$PWD/hpg-fastq_amd/libhpgq.so; else L=$PWD/hpg-fastq_amd/ab/libhpgq_peov0.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config c4_pe --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_c4_pe_$v.jsonl 2>> $O/bench.err || exit 4
done
