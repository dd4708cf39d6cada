# Kernel-time A/B of library variants on prof_engine.py modes (rocprofv3
# kernel trace; one run per variant and mode, variants alternating).
#   TAG=... VARIANTS="name=lib ..." MODES="mode:reads:L ..." REPS=2 bash tools/kstat_ab.sh
# -> gpurun_out/$TAG/kstat_<name>_<mode>_<rep>/ (the kernel_stats CSV)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-kstat}
mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for spec in $MODES; do
    IFS=: read mode n L <<< "$spec"
    for v in $VARIANTS; do
      name=${v%%=*}; lib=${v#*=}
      if [ "$lib" = . ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/$lib; fi
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kstat_${name}_${mode}_$r -o run --output-format csv -- python3 tools/prof_engine.py --mode $mode --reads $n --L $L --iters 5 > $O/kstat_${name}_${mode}_$r.log 2>&1 || exit 4
    done
  done
done
unset HPGQ_LIB_PATH
echo done > $O/DONE
