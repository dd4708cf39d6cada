# round 3 A/B on one box: HEAD's libhpgq (hpg-fastq_amd/ab/head) vs the working tree,
# bench lines of CFGS alternating A B A B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in head new; do
    for c in ${CFGS:-c2 c3 c4}; do
      if [ $v = head ]; then export HPGQ_LIB_PATH=$GRAFT_REPO_ROOT/hpg-fastq_amd/ab/head/libhpgq.so; else unset HPGQ_LIB_PATH; fi
      timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/ab/$v.$c.$rep.json 2> gpurun_out/ab/$v.$c.$rep.err || { tail -5 gpurun_out/ab/$v.$c.$rep.err; exit 2; }
      python -c "import json; d=json.load(open('gpurun_out/ab/$v.$c.$rep.json')); r=d['roofline']; print('$rep $v $c', r['avg_launch_us'], r['frac'])"
    done
  done
done
