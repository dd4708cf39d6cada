#!/bin/bash
# round 4: where filter / edit spend their time end to end (HPGQ_TRACE=1:
# per chunk read / parse / sync / placement / copy times), 10 M reads in /dev/shm
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t
mkdir -p $O
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_t || exit 4
F=/dev/shm/hpgq_e2et.fq
D=/dev/shm/hpgq_e2et_out
timeout -k 10 300 /tmp/fqgen_t $F 10000000 150 2 || { rm -f $F; exit 5; }
mkdir -p $D
for cmd in stats filter edit; do
  ex=""
  [ $cmd = edit ] && ex="--left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20,"
  [ $cmd != edit ] && ex="--read-quality-range 20, --read-length-range 50,"
  for rep in 1 2; do
    rm -rf $D/*
    HPGQ_TRACE=1 timeout -k 10 300 hpg-fastq_amd/hpg-fastq $cmd -f $F -o $D $ex --num-threads 16 --gpus 1 > $O/${cmd}_$rep.log 2> $O/${cmd}_$rep.trace || { rm -rf $F $D; exit 6; }
  done
done
# the same with the output files symlinked to /dev/null (no page-cache
# allocation: the pipeline without the file system's write)
for cmd in filter edit; do
  ex="--read-quality-range 20, --read-length-range 50,"
  [ $cmd = edit ] && ex="--left-length 10 --left-quality-range 20, --right-length 30 --right-quality-range 20,"
  for rep in 1 2; do
    rm -rf $D/*
    ln -s /dev/null $D/passed.fq; ln -s /dev/null $D/failed.fq; ln -s /dev/null $D/edit.fq
    HPGQ_TRACE=1 timeout -k 10 300 hpg-fastq_amd/hpg-fastq $cmd -f $F -o $D $ex --num-threads 16 --gpus 1 > $O/${cmd}_devnull_$rep.log 2> $O/${cmd}_devnull_$rep.trace || { rm -rf $F $D; exit 7; }
  done
done
cat /sys/kernel/mm/transparent_hugepage/shmem_enabled > $O/thp.txt 2>&1; uname -r >> $O/thp.txt
nproc > $O/nproc.txt; cat /proc/self/status | grep -i cpus_allowed_list >> $O/nproc.txt
rm -rf $F $D /tmp/fqgen_t
