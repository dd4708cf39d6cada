#!/bin/bash
# round 4, call C: pipeline trace (filter / edit e2e), same-box A/B of the
# spill fixes (HPGQ_TAB_LEN / HPGQ_FX_LDS; ab/r3base = round 3's layout) on
# the engine configs, the drop-in harness, then the C5 ablation
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_dropin_gpu.py tests/test_engine_gpu.py -k "writer or outputs or tsan or dropin or read_counters or route or host" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 6
bash tools/gpu_r04_trace.sh || exit $?
for cfg in c2 c3 c4 c4_pe c4_noor; do
  for v in new base new base; do
    if [ $v = base ]; then L=$PWD/hpg-fastq_amd/ab/r3base/libhpgq.so; else L=$PWD/hpg-fastq_amd/libhpgq.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline >> $O/bench_${cfg}_$v.jsonl 2>> $O/bench.err || exit 7
  done
done
timeout -k 10 400 python bench.py --config dropin --steps 5 > $O/dropin.json 2> $O/dropin.err || exit 8
# one no-sync worker alone under the kernel + copy trace (the H2D rate of one ctx's staging DMA)
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_d && timeout -k 10 120 /tmp/fqgen_d /dev/shm/hpgq_dtr.fq 2000000 150 2 || exit 9
for t in 1 2 4; do
  timeout -k 10 120 ./tools/dropin_bench /dev/shm/hpgq_dtr.fq --threads $t --c2 --lmax 1024 --repeat 5 --no-sync >> $O/dropin_sweep.jsonl 2>> $O/dropin.err || { rm -f /dev/shm/hpgq_dtr.fq; exit 10; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/dtrace1 -o run --output-format csv -- ./tools/dropin_bench /dev/shm/hpgq_dtr.fq --threads 1 --c2 --lmax 1024 --repeat 3 --no-sync > $O/dtrace1.json 2> $O/dtrace1.err || { rm -f /dev/shm/hpgq_dtr.fq; exit 11; }
rm -f /dev/shm/hpgq_dtr.fq
# (the C5 ablation runs in its own call: tools/gpu_c5_ablation_r04.sh)
