# c1_wgrad with two tile groups per block: op tests, the critic first-layer wgrad case (1 vs 2
# groups), bench, and a plan-mode kernel trace for the step timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4h_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4h_ops.log; exit 1; }
timeout -k 10 200 python -u tools/bench_ops.py --case crit_first_wgrad --tune 18=1,2 > gpurun_out/r4h_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_dgrad_k3m >> gpurun_out/r4h_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case res_wgrad_k3m --tune 19=0,8,1,2,4,3 >> gpurun_out/r4h_probe.txt 2>&1 || exit $?
CGAN3D_TUNE=16=2 timeout -k 10 200 python -u tools/bench_ops.py --case res_wgrad_k3m --tune 19=0,8,1,2,4 >> gpurun_out/r4h_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4h_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4h_step.log
for i in 1 2; do timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4h_bench_$i.json 2>/dev/null || exit $?; done
CGAN3D_TUNE=18=1 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4h_bench_g1.json 2>/dev/null || exit $?
CGAN3D_TUNE=16=2 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4h_bench_k9m.json 2>/dev/null || exit $?
timeout -k 10 150 python -u tools/plan_host_time.py > gpurun_out/r4h_host.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r4h_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4h_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $R/gpurun_out/r4h_trace.json 2> $R/gpurun_out/r4h_trace.err
