# round 3: full GPU suite, bench, rocprof kernel trace of the bench (plan mode)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=15 --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
CGAN3D_FORCE_DP=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dp1.json 2> gpurun_out/bench_dp1.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace_main -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/trace_main.json 2> $GRAFT_REPO_ROOT/gpurun_out/trace_main.err || exit $?
exit $rc
