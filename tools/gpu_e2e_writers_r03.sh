# round 3: CLI end to end for the subcommands that WRITE FastQ (filter: passed /
# failed files, edit: the trimmed file) beside stats, on one synthetic file in
# /dev/shm (input and outputs in memory: the reader, GPU and writer are timed,
# not a disk)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2ew
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_w || exit 4
F=/dev/shm/hpgq_e2ew.fq
O=/dev/shm/hpgq_e2ew_out
N=${N:-10000000}
timeout -k 10 300 /tmp/fqgen_w $F $N 150 2 || { rm -f $F; exit 5; }
mkdir -p $O
run() {   # name, args...
  local name=$1; shift
  for rep in 1 2 3; do
    rm -rf $O/*
    local t0=$(date +%s.%N)
    timeout -k 10 300 hpg-fastq_amd/hpg-fastq "$@" -f $F -o $O --num-threads 16 --gpus 1 > gpurun_out/e2ew/${name}_r$rep.log 2>&1 || { rm -rf $F $O; exit 6; }
    local t1=$(date +%s.%N)
    python3 -c "import sys; t=$t1-$t0; print('$name', $rep, round(t,3), 's', round($N/t/1e6,1), 'Mreads/s')" | tee -a gpurun_out/e2ew/summary.txt
  done
  ls -la $O >> gpurun_out/e2ew/${name}_files.txt
}
run stats stats --read-quality-range 20, --read-length-range 50,
run filter filter --read-quality-range 20, --read-length-range 50,
run edit edit --left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20,
rm -rf $F $O /tmp/fqgen_w
