# round 3 A/B on one box: libhpgq variants under hpg-fastq_amd/ab/<name> (VARIANTS;
# "base" = the working tree's build), bench lines of CFGS, REPS rounds alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-base head}; do
    for c in ${CFGS:-c2 c3 c4}; do
      if [ $v = base ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$GRAFT_REPO_ROOT/hpg-fastq_amd/ab/$v/libhpgq.so; fi
      timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/ab/$v.$c.$rep.json 2> gpurun_out/ab/$v.$c.$rep.err || { tail -5 gpurun_out/ab/$v.$c.$rep.err; exit 2; }
      python -c "import json; d=json.load(open('gpurun_out/ab/$v.$c.$rep.json')); r=d['roofline']; print('$rep $v $c', r['avg_launch_us'], r['frac'])"
    done
  done
done
