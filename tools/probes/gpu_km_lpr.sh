# probe: kmer_tile_kernel one vs two lanes per read (id-major conflict-free table): tests, timing, HBM bytes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kmlpr
export TMPDIR=/tmp
for L in 1 2; do
  HPGQ_KMERS_LPR=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kmers_gpu.py > gpurun_out/kmlpr/tests_$L.log 2>&1 || { tail -30 gpurun_out/kmlpr/tests_$L.log; exit 1; }
  tail -1 gpurun_out/kmlpr/tests_$L.log
  HPGQ_KMERS_LPR=$L timeout -k 10 300 python bench.py --config c2_kmers --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/kmlpr/bench_$L.json 2> gpurun_out/kmlpr/bench_$L.err || { tail -5 gpurun_out/kmlpr/bench_$L.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/kmlpr/bench_$L.json')); r=d['roofline']; print('lpr $L', d['value'], r['avg_launch_us'], r['frac'])"
  HPGQ_KMERS_LPR=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/kmlpr/fetch_$L -o run --output-format csv -- python tools/prof_engine.py --mode c2 --kmers --iters 2 > gpurun_out/kmlpr/fetch_$L.log 2>&1 || exit 3
done
