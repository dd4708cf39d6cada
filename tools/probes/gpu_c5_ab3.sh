# probe: C5 stream kernel A/B on one box: committed (ab/base), register start bits (tree), LDS bitmap
# without the read back (ab/noso, timing only); all reads and 5 % skipped
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5ab
export TMPDIR=/tmp
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 8"
for M in cgr cgrv; do
  for V in base tree noso; do
    if [ $V = tree ]; then L=""; else L=$PWD/hpg-fastq_amd/ab/$V/libhpgq.so; fi
    if [ $V = noso ] && [ $M = cgrv ]; then continue; fi
    HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5ab/${V}_$M -o run --output-format csv -- $A --mode $M > gpurun_out/c5ab/${V}_$M.log 2>&1 || exit 1
  done
done
