# BatchNorm accumulators (apply mode) + merged generator-loss pass: parity subset, kernel trace, A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_api.py \
  -k "accumulators or plan_replay or fixture or zncc or loss or shadows" > gpurun_out/fuse2_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k "bf16 and 64" > gpurun_out/fuse2_cfg.log 2>&1 || exit $?
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/f2_apply_$k.json 2> gpurun_out/f2_apply_$k.err || exit $?
CGAN3D_NO_BN_FUSE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/f2_off_$k.json 2> gpurun_out/f2_off_$k.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/tf2
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tf2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/tf2.json 2> $GRAFT_REPO_ROOT/gpurun_out/tf2.err
