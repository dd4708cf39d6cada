# round 3 final (gpurun): the whole GPU suite, then the profile set (tools/gpu_profile_r03.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03/gpu_suite.log 2>&1 || { echo SUITE_FAILED; grep -E "FAILED|Error|error" gpurun_out/r03/gpu_suite.log | head -20; tail -30 gpurun_out/r03/gpu_suite.log; exit 1; }
tail -1 gpurun_out/r03/gpu_suite.log
bash tools/gpu_profile_r03.sh
