set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
for v in main nt1 nt2; do
  L=""; [ $v != main ] && L=hpg-fastq_amd/ab/$v/libhpgq.so
  for c in c4 c4_pe; do
    HPGQ_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/aux_${v}_$c.json 2>/dev/null || exit 2
    python -c "import json; d=json.load(open('gpurun_out/r03/aux_${v}_$c.json')); r=d['roofline']; print('$v $c', d['value'], r['avg_launch_us'], r['frac'])"
  done
  HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcaux_$v -o run --output-format csv -- python tools/prof_engine.py --mode edit --reads 12500000 --iters 2 > /dev/null 2>&1 || exit 3
done
