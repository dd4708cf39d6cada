# engine tests + C2/C4 bench: hex (default) vs tri geometry (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/geo
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/geo/test.log 2>&1 || exit 3
for i in 1 2; do
for geo in hex tri; do
  for c in ${CFGS:-c2 c4}; do
    HPGQ_TRI_GEO=$geo timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/geo/bench_${geo}_${c}_$i.json 2> gpurun_out/geo/bench_${geo}_${c}_$i.err || exit 4
  done
done
done
