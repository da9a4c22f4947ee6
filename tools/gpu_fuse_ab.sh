# BatchNorm through fp64 accumulators (cgan3d_bn_fuse): parity tests, then bench A/B of the modes
# (CGAN3D_BN_ACC apply / stage, CGAN3D_NO_BN_FUSE=1 slabs), two rounds each, back to back on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py \
  -k "fused_resnet or plan_replay or shadows_match or folded_last or fixture" > gpurun_out/fuse_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k "bf16 and 64" > gpurun_out/fuse_cfg.log 2>&1 || exit $?
for k in 1 2; do
CGAN3D_BN_ACC=apply timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fuse_apply_$k.json 2> gpurun_out/fuse_apply_$k.err || exit $?
CGAN3D_BN_ACC=stage timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fuse_stage_$k.json 2> gpurun_out/fuse_stage_$k.err || exit $?
CGAN3D_NO_BN_FUSE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/fuse_off_$k.json 2> gpurun_out/fuse_off_$k.err || exit $?
done
