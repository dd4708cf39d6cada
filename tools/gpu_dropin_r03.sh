# round 3: the host-path tests (in-place staging), then the drop-in bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dropin
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dropin_gpu.py tests/test_abi_cpu.py > gpurun_out/dropin/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/dropin/tests.log | head -30; tail -30 gpurun_out/dropin/tests.log; exit 1; }
tail -1 gpurun_out/dropin/tests.log
timeout -k 10 300 python bench.py --config dropin > gpurun_out/dropin/bench_dropin.json 2> gpurun_out/dropin/bench_dropin.err || { tail -20 gpurun_out/dropin/bench_dropin.err; exit 2; }
cat gpurun_out/dropin/bench_dropin.json
# the harness at 1 / 2 / 4 worker threads, in place and copied
gcc -O2 -fopenmp tools/fqgen.c -o /tmp/fqgen_$$ && /tmp/fqgen_$$ /dev/shm/hpgq_dropin_sweep.fq 4000000 150 2 || exit 3
for t in 1 2 4; do
  for mode in "" "--copy"; do
    timeout -k 10 120 ./tools/dropin_bench /dev/shm/hpgq_dropin_sweep.fq --threads $t --c2 --lmax 1024 --repeat 5 $mode | tee -a gpurun_out/dropin/sweep.log || { rm -f /dev/shm/hpgq_dropin_sweep.fq; exit 4; }
  done
done
rm -f /dev/shm/hpgq_dropin_sweep.fq /tmp/fqgen_$$
