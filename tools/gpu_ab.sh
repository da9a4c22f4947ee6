# A/B of an env switch (AB="VAR=value"): selected tests, then bench with and without the switch
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${FILES:-tests/test_gpu_ops.py} -x -q -k "${TESTS:-halo}" --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || exit $?
env $AB timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_a2.json 2> gpurun_out/bench_a2.err
