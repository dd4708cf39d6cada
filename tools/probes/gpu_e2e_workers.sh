# CLI end to end with 1..3 GPU workers on one GPU (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2ew
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen || exit 4
timeout -k 10 300 /tmp/fqgen /tmp/e2e.fq ${N:-20000000} 150 2 > gpurun_out/e2ew/gen.log 2>&1 || exit 5
mkdir -p /tmp/e2e_out
for g in ${GPUS:-1 2 3}; do
  for rep in 1 2 3; do
    timeout -k 10 300 hpg-fastq_amd/hpg-fastq stats -f /tmp/e2e.fq -o /tmp/e2e_out --read-quality-range 20, --read-length-range 50, --num-threads 16 --gpus $g --chunk-mb ${CHUNK:-256} > gpurun_out/e2ew/g${g}_r${rep}.log 2>&1 || exit 6
  done
done
rm -f /tmp/e2e.fq
