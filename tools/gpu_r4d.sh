# conv_k3m after the epilogue-operand prefetch: op tests, the phase probe, the step tests, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "k3m or halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4d_ops.log; exit 1; }
timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_dgrad_k3m --tune 17=0,1,2,3,4,8,7,15 > gpurun_out/r4d_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4d_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4d_step.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4d_bench_$i.json 2>/dev/null || exit $?; done
