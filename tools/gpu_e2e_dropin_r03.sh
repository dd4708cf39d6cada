set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 500 python bench.py > gpurun_out/r03/bench_default2.json 2> gpurun_out/r03/bench_default2.err || { tail -20 gpurun_out/r03/bench_default2.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/r03/bench_default2.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['e2e']))"
timeout -k 10 300 python bench.py --config dropin --steps 5 > gpurun_out/r03/bench_dropin.json 2> gpurun_out/r03/bench_dropin.err || { tail -20 gpurun_out/r03/bench_dropin.err; exit 3; }
cat gpurun_out/r03/bench_dropin.json
