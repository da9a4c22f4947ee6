# Round-4 kernel changes (resident halo weight slabs, critic last-layer kernels, c1 / sk epilogue
# prefetch): op and step tests, the default bench twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4j_ops.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4j_step.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4j_bench_$i.json 2>/dev/null || exit $?; done
