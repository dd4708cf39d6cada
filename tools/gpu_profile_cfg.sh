# one or more configs' profile records (gpurun): a traced bench line and the
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE, one per run) on the same kernels and
# batch, as tools/gpu_profile_r03.sh does per config.  SPECS as there.
# Then: python tools/profile_report.py --round r03 --prof gpurun_out/profc
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/profc
mkdir -p $P
for spec in ${SPECS:-c2_noor:maxn:10000000:150}; do
  IFS=: read cfg mode n L extra <<< "$spec"
  A="python tools/prof_engine.py --mode $mode --reads $n --L $L --iters 3 $extra"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/btrace_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > $P/bench_$cfg.json 2> $P/bench_$cfg.err || exit 4
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/fetch_$cfg -o run --output-format csv -- $A > $P/fetch_$cfg.log 2>&1 || exit 5
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/write_$cfg -o run --output-format csv -- $A > $P/write_$cfg.log 2>&1 || exit 6
  cat $P/bench_$cfg.json
done
