# Cross-stream waits bound to the waited-on launch's completion event: step tests, then bench A/B
# against CGAN3D_DEBUG=event_record (a marker event per wait), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4f_step.log
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4f_bench_bind_$i.json 2>/dev/null || exit $?
  CGAN3D_DEBUG=event_record timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4f_bench_rec_$i.json 2>/dev/null || exit $?
done
