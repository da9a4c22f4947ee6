# GPU step tests (bf16 configurations), two default bench runs and a plan-mode kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_step.py -k "${BT_TESTS:-(bf16 and 64) or plan_replay or accumulators or fixture}" > gpurun_out/bt_tests.log 2>&1 || exit $?
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bt_$k.json 2> gpurun_out/bt_$k.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/bt_trace
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bt_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bt_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/bt_trace.err
