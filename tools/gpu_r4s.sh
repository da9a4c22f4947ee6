# The critic first-layer weight grad at 8 tiles per block by default: op and step tests, bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/r4s_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err || exit $?
