#!/bin/bash
# round 4: name C5's bound.  Timing-only variants of
# cgr_stream_kernel<7> (HPGQ_C5_ABLATION, hpgq_cgr_stream.h; built by
# tools/probes/build_cgr_ab.sh c5abl<v> -DHPGQ_C5_ABLATION=<v>):
#   base  the product kernel
#   1     no table add (VALU xor instead of ds_add_u64)
#   2     quality window chain -> constant
#   3     no emission mask
#   4     ds_add_u32 of the count only
# per variant: bench --config c5 (HIP-event time per launch) and one PMC pass
# of 7 counters on tools/prof_engine.py --mode cgr.  Summary:
# python tools/c5_ablation_report.py gpurun_out/c5abl > profiles/r04_c5_ablation.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/c5abl
mkdir -p $D
for v in base 1 2 3 4 5; do
  if [ $v = base ]; then LIB=$PWD/hpg-fastq_amd/libhpgq.so; else LIB=$PWD/hpg-fastq_amd/ab/libhpgq_c5abl$v.so; fi
  for rep in 1 2; do
    HPGQ_LIB_PATH=$LIB HPGQ_BENCH_NOCHECK=1 timeout -k 10 180 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $D/bench_${v}_$rep.json 2> $D/bench_${v}_$rep.err || exit 3
  done
  HPGQ_LIB_PATH=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $D/pmc_$v -o run --output-format csv -- python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 2 > $D/pmc_$v.log 2>&1 || exit 4
  HPGQ_LIB_PATH=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $D/pmc2_$v -o run --output-format csv -- python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 2 > $D/pmc2_$v.log 2>&1 || exit 5
done
# the exact variant 5 (EXEC-masked adds) against the product on ONLY_VALID_READS, where ~7 % of
# the bytes end no word (5 % skipped reads + read starts)
for v in base 5 base 5; do
  if [ $v = base ]; then LIB=$PWD/hpg-fastq_amd/libhpgq.so; else LIB=$PWD/hpg-fastq_amd/ab/libhpgq_c5abl$v.so; fi
  HPGQ_LIB_PATH=$LIB timeout -k 10 180 python bench.py --config c5_valid --steps 10 --warmup 3 --no-cpu-baseline >> $D/bench_valid_$v.jsonl 2>> $D/bench_valid.err || exit 6
done
