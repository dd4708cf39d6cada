# round 3: kernel + copy trace of the drop-in worker (2 threads, in place) -- where a
# 10,000-read batch's GPU time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dtrace
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_d || exit 3
/tmp/fqgen_d /dev/shm/hpgq_dtrace.fq 2000000 150 2 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/dtrace/t -o run --output-format csv -- ./tools/dropin_bench /dev/shm/hpgq_dtrace.fq --threads 2 --c2 --lmax 1024 --repeat 3 > gpurun_out/dtrace/harness.json 2> gpurun_out/dtrace/err.log || { rm -f /dev/shm/hpgq_dtrace.fq; exit 5; }
rm -f /dev/shm/hpgq_dtrace.fq /tmp/fqgen_d
cat gpurun_out/dtrace/harness.json
find gpurun_out/dtrace/t -name "*stats.csv" | head
for f in $(find gpurun_out/dtrace/t -name "*_stats.csv"); do echo "== $f"; cut -d, -f1-6 $f | head -12; done
