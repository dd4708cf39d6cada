# probe: hex units of 24 reads instead of 48 (ab/blk24) vs the tree: C2, C4, c4_pe, c4_noor kernel time and
# HBM bytes (shorter reuse distance for the edit prologue's trim lines)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/blk
export TMPDIR=/tmp
for spec in c2:c2:10000000 edit:edit:12500000 pe_edit:pe_edit:10000000; do
  IFS=: read name mode n <<< "$spec"
  A="python tools/prof_engine.py --mode $mode --reads $n --iters 6"
  for V in tree blk24; do
    if [ $V = tree ]; then L=""; else L=$PWD/hpg-fastq_amd/ab/$V/libhpgq.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/blk/${V}_$name -o run --output-format csv -- $A > gpurun_out/blk/${V}_$name.log 2>&1 || exit 1
    HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/blk/f_${V}_$name -o run --output-format csv -- $A > gpurun_out/blk/f_${V}_$name.log 2>&1 || exit 2
  done
done
