# quick GPU iteration: selected tests (TESTS, pytest -k expression), host timing, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${FILES:-tests/test_gpu_ops.py tests/test_gpu_step.py} -x -q -k "${TESTS:-plan}" --timeout 120 --timeout-method thread > gpurun_out/quick_test.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/host_time.py > gpurun_out/host_time.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
