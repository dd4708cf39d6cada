set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "edit or paired" > gpurun_out/r03/edit_tests.log 2>&1 || { tail -20 gpurun_out/r03/edit_tests.log; exit 1; }
tail -1 gpurun_out/r03/edit_tests.log
for spec in main:c4 main:c4_noor main:c4_pe tri:c4_pe tri:c3 main:c3; do
  v=${spec%%:*}; c=${spec##*:}
  G=""; [ $v = tri ] && G=tri
  HPGQ_TRI_GEO=$G timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/ab_${v}_$c.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/r03/ab_${v}_$c.json')); r=d['roofline']; print('$v $c', d['value'], r['avg_launch_us'], r['frac'], r['kernel'])"
done
