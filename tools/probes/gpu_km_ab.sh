set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03 gpurun_out/pmckm
export TMPDIR=/tmp
for v in main km2; do
  L=""; [ $v != main ] && L=hpg-fastq_amd/ab/$v/libhpgq.so
  HPGQ_LIB_PATH=$L timeout -k 10 300 python bench.py --config c2_kmers --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03/km_$v.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/r03/km_$v.json')); r=d['roofline']; print('$v', d['value'], r['avg_launch_us'], r['frac'])"
  A="python tools/prof_engine.py --mode c2 --kmers --iters 2"
  HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmckm_$v/fetch -o run --output-format csv -- $A > /dev/null 2>&1 &&
  HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE TA_BUFFER_READ_WAVEFRONTS_sum -d gpurun_out/pmckm_$v/ta -o run --output-format csv -- $A > /dev/null 2>&1 &&
  HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d gpurun_out/pmckm_$v/p2 -o run --output-format csv -- $A > /dev/null 2>&1 || exit 3
done
