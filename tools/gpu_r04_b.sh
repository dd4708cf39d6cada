#!/bin/bash
# round 4: the mapped parallel writer (filter / edit) — CLI byte-compare tests
# (both writers, edges, TSan), then end to end on one synthetic file in
# /dev/shm (input and outputs in memory), mapped vs stream writer, 3 runs each
# (CLI-internal clock = its Throughput line, plus wall time)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread > $O/cli_tests.log 2>&1 || exit 3
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_w || exit 4
F=/dev/shm/hpgq_e2ew.fq
D=/dev/shm/hpgq_e2ew_out
N=${N:-10000000}
timeout -k 10 300 /tmp/fqgen_w $F $N 150 2 || { rm -f $F; exit 5; }
mkdir -p $D
run() {   # name, args...
  local name=$1; shift
  for rep in 1 2 3; do
    rm -rf $D/*
    local t0=$(date +%s.%N)
    timeout -k 10 300 hpg-fastq_amd/hpg-fastq "$@" -f $F -o $D --num-threads 16 --gpus 1 > $O/${name}_r$rep.log 2>&1 || { rm -rf $F $D; exit 6; }
    local t1=$(date +%s.%N)
    local tp=$(grep -o "= [0-9.]* Mreads/s" $O/${name}_r$rep.log)
    echo "$name $rep wall $(python3 -c "print(round($t1-$t0,3))") s, CLI $tp" | tee -a $O/summary.txt
  done
  ls -la $D >> $O/${name}_files.txt
}
run stats stats --read-quality-range 20, --read-length-range 50,
run filter filter --read-quality-range 20, --read-length-range 50,
run filter_stream filter --read-quality-range 20, --read-length-range 50, --stream-writer
run edit edit --left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20,
run edit_stream edit --left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20, --stream-writer
run edit_filter edit --left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20, --read-quality-range 20,
rm -rf $F $D /tmp/fqgen_w
