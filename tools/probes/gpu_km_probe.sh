set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
for v in ${VS:-main kmp1 kmp2 kmp3}; do
  L=""; [ $v != main ] && L=hpg-fastq_amd/ab/$v/libhpgq.so
  HPGQ_BENCH_NOCHECK=1 HPGQ_LIB_PATH=$L timeout -k 10 300 python bench.py --config c2_kmers --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03/km_$v.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/r03/km_$v.json')); r=d['roofline']; print('$v', d['value'], r['avg_launch_us'], r['frac'])"
done
