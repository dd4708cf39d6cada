# One parameterised GPU session (run via gpurun), replacing the per-call
# one-off scripts of rounds 3-4.  Every step has its own time limit and the
# session stops at the first failing step.  Environment:
#   TAG       output directory gpurun_out/$TAG                       (default run)
#   TESTS     pytest -k expression for the GPU suite; "all" = whole suite; empty = none
#   VARIANTS  "name=path/to/libhpgq.so ..." (name=. : the in-tree build) (default base=.)
#   CFGS      bench configs timed per variant                        (default none)
#   REPS      alternating rounds over the variants                    (default 2)
#   STEPS     bench --steps (default 10)
#   PMC       "cfg:mode:reads:L[:extra] ..." FETCH_SIZE / WRITE_SIZE passes per variant
#             on tools/prof_engine.py (one counter per pass)
#   SQ        "cfg:mode:reads:L[:extra] ..." SQ instruction-mix passes (in-tree build)
#   TRACE     1: rocprofv3 kernel trace of each variant's bench runs (first round)
# Summarise with: python tools/ab_summary.py gpurun_out/$TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p $O
if [ -n "$TESTS" ]; then
  if [ "$TESTS" = all ]; then K=(); else K=(-k "$TESTS"); fi
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1 || exit 3
fi
VARIANTS=${VARIANTS:-base=.}
for r in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    name=${v%%=*}; lib=${v#*=}
    if [ "$lib" = . ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/$lib; fi
    for c in $CFGS; do
      if [ "$r" = 1 ] && [ -n "$TRACE" ]; then
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_${name}_$c -o run --output-format csv -- python3 bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline >> $O/bench_${name}_$c.jsonl 2>> $O/bench.err || exit 4
      else
        timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline >> $O/bench_${name}_$c.jsonl 2>> $O/bench.err || exit 4
      fi
    done
  done
done
for v in $VARIANTS; do
  name=${v%%=*}; lib=${v#*=}
  if [ "$lib" = . ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/$lib; fi
  for spec in $PMC; do
    IFS=: read cfg mode n L extra <<< "$spec"
    A="python tools/prof_engine.py --mode $mode --reads $n --L $L --iters 3 $extra"
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${name}_${cfg}_$ctr -o run --output-format csv -- $A > $O/pmc_${name}_${cfg}_$ctr.log 2>&1 || exit 5
    done
  done
done
# SQ passes: the in-tree build, or every variant with SQVAR=1 (sq1_<name>_<cfg>)
for v in $([ -n "$SQVAR" ] && echo $VARIANTS || echo "base=."); do
  name=${v%%=*}; lib=${v#*=}
  if [ "$lib" = . ]; then unset HPGQ_LIB_PATH; else export HPGQ_LIB_PATH=$PWD/$lib; fi
  tag=$([ -n "$SQVAR" ] && echo "${name}_" || echo "")
  for spec in $SQ; do
    IFS=: read cfg mode n L extra <<< "$spec"
    A="python tools/prof_engine.py --mode $mode --reads $n --L $L --iters 3 $extra"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d $O/sq1_$tag$cfg -o run --output-format csv -- $A > $O/sq1_$tag$cfg.log 2>&1 || exit 6
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $O/sq2_$tag$cfg -o run --output-format csv -- $A > $O/sq2_$tag$cfg.log 2>&1 || exit 6
  done
done
unset HPGQ_LIB_PATH
echo done > $O/DONE
