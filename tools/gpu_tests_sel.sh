# selected GPU tests (FILES, TESTS = pytest -k expression), then the default bench line
#   FILES="tests/test_gpu_configs.py" TESTS="bf16" gpurun -- bash tools/gpu_tests_sel.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -v -k "${TESTS:-gpu}" --timeout 240 --timeout-method thread --durations=20 > gpurun_out/sel_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/sel_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
