# CLI end-to-end FASTQ-file throughput (run via gpurun): the drop-in default
# (no --lmax: 1024) beside --lmax 150, several reader-thread counts
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen || exit 4
N=${N:-20000000}
( time timeout -k 10 300 /tmp/fqgen /tmp/e2e.fq $N 150 2 ) > gpurun_out/e2e/gen.log 2>&1 || exit 5
ls -la /tmp/e2e.fq >> gpurun_out/e2e/gen.log
mkdir -p /tmp/e2e_out
for t in ${THREADS:-16}; do
  for lm in default 150; do
    LM=""; [ "$lm" != default ] && LM="--lmax $lm"
    for rep in 1 2 3; do
      timeout -k 10 300 hpg-fastq_amd/hpg-fastq stats -f /tmp/e2e.fq -o /tmp/e2e_out --read-quality-range 20, --read-length-range 50, $LM --num-threads $t --chunk-mb ${CHUNK:-256} ${E2E_ARGS} > gpurun_out/e2e/stats_t${t}_lmax${lm}_r${rep}.log 2>&1 || exit 6
    done
  done
done
cp /tmp/e2e_out/e2e.fq.summary.txt gpurun_out/e2e/ 2>/dev/null
rm -f /tmp/e2e.fq
