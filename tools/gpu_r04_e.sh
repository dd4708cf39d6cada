#!/bin/bash
# round 4, call E: CGR stream kernel with three tiles of bytes in flight per
# wave (HPGQ_C5_DEPTH 3, the product) against two (ab/libhpgq_d2.so): CGR
# parity tests, then C5 / C5-valid bench A/B and one PMC pass each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 3
for v in d3 d2 d3 d2 d3 d2; do
  if [ $v = d2 ]; then L=$PWD/hpg-fastq_amd/ab/libhpgq_d2.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_$v.jsonl 2>> $O/bench.err || exit 4
done
for v in d3 d2; do
  if [ $v = d2 ]; then L=$PWD/hpg-fastq_amd/ab/libhpgq_d2.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
  HPGQ_LIB_PATH=$L timeout -k 10 180 python bench.py --config c5_valid --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_valid_$v.jsonl 2>> $O/bench.err || exit 5
  HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$v -o run --output-format csv -- python tools/prof_engine.py --mode cgr --reads 5000000 --L 250 --iters 2 > $O/pmc_$v.log 2>&1 || exit 6
done
