# Branch-free c1 staging / epilogues, bf16 ResNet storage: op tests, critic cases, step tests, bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4i_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4i_ops.log; exit 1; }
timeout -k 10 200 python -u tools/bench_ops.py --case crit_first crit_first_wgrad crit_m0 crit_m1 crit_m2 res_wgrad_k3m > gpurun_out/r4i_probe.txt 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4i_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4i_step.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4i_bench_$i.json 2>/dev/null || exit $?; done
CGAN3D_DEBUG=fp32_store timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4i_bench_fp32store.json 2>/dev/null || exit $?
for v in 128 256; do
  CGAN3D_TUNE=20=$v timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4i_bench_k7wg$v.json 2>/dev/null || exit $?
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4i_bench_def$v.json 2>/dev/null || exit $?
done
