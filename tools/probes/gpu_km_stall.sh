# probe: kmer_tile_kernel stall counters for one and two lanes per read
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kmstall
export TMPDIR=/tmp
for L in 1 2; do
  HPGQ_KMERS_LPR=$L timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES -d gpurun_out/kmstall/a_$L -o run --output-format csv -- python tools/prof_engine.py --mode c2 --kmers --iters 2 > gpurun_out/kmstall/a_$L.log 2>&1 || exit 1
  HPGQ_KMERS_LPR=$L timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_LDS -d gpurun_out/kmstall/b_$L -o run --output-format csv -- python tools/prof_engine.py --mode c2 --kmers --iters 2 > gpurun_out/kmstall/b_$L.log 2>&1 || exit 2
done
