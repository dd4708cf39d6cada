# CLI end-to-end runs with the per-chunk trace (HPGQ_TRACE=1), to find where a
# slow run spends its time (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2et
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen || exit 4
timeout -k 10 300 /tmp/fqgen /tmp/e2e.fq ${N:-20000000} 150 2 > gpurun_out/e2et/gen.log 2>&1 || exit 5
mkdir -p /tmp/e2e_out
for rep in $(seq 1 ${REPS:-10}); do
  HPGQ_TRACE=1 timeout -k 10 300 hpg-fastq_amd/hpg-fastq stats -f /tmp/e2e.fq -o /tmp/e2e_out --read-quality-range 20, --read-length-range 50, --num-threads 16 > gpurun_out/e2et/r$rep.log 2>&1 || exit 6
done
rm -f /tmp/e2e.fq
