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
# (the C5 ablation runs in its own call: tools/gpu_c5_ablation_r04.sh)
