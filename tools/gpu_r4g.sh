# LDS-only barriers in the epilogues / prefetch pipelines: op tests, k3m cases, step tests, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bn_fused.py tests/test_gpu_2d.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4g_ops.log; exit 1; }
timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_dgrad_k3m > gpurun_out/r4g_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4g_step.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4g_bench_$i.json 2>/dev/null || exit $?; done
