# run a pytest selection on the GPU box (via gpurun): TESTS="tests/test_x.py -k y"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${T:-600} python -m pytest ${TESTS:-tests} -x -q -m gpu > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_sel.log
exit $rc
