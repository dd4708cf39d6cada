# One gpurun session: a list of GPU test files, then tools/gpu_run.sh's A/B
# benches (TAG, VARIANTS, CFGS, REPS, STEPS as there).  Every step has its own
# time limit; the session stops at the first failing step.
#   PYTESTS="tests/a.py tests/b.py" TAG=x VARIANTS="..." CFGS="c2 c4" bash tools/gpu_session.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p $O
if [ -n "$PYTESTS" ]; then
  timeout -k 10 ${PYTIME:-900} python -u -m pytest $PYTESTS -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || [ -n "$CONTINUE_ON_FAIL" ] || exit 3
  case $rc in 0|1) ;; *) exit 3 ;; esac
fi
[ -n "$CFGS$PMC$SQ" ] || exit 0
TESTS= bash tools/gpu_run.sh
