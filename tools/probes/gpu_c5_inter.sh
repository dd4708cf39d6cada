# probe: C5 with the next tile's classification spread over this tile's adds (tree) vs the committed kernel
# (ab/base): CGR tests, then timing (all reads, 5 % skipped) and bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5i gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cgr_gpu.py tests/test_cgr_fuzz_gpu.py > gpurun_out/r03/cgr_tests.log 2>&1 || { tail -30 gpurun_out/r03/cgr_tests.log; exit 1; }
tail -1 gpurun_out/r03/cgr_tests.log
A="python tools/prof_engine.py --reads 5000000 --L 250 --iters 8"
for M in cgr cgrv; do
  for V in base tree; do
    if [ $V = tree ]; then L=""; else L=$PWD/hpg-fastq_amd/ab/$V/libhpgq.so; fi
    HPGQ_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5i/${V}_$M -o run --output-format csv -- $A --mode $M > gpurun_out/c5i/${V}_$M.log 2>&1 || exit 2
  done
done
