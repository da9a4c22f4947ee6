# Same-box A/B of the current library (halo ring and critic k4 kernel restored; critic last-layer
# kernels, folded BatchNorm backward and accumulator-pass trips kept) against the r4i-verified build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
OLD=$R/contrast-gan-3d_amd/ab/libcgan3d_e4d2.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4l_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4l_ops.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4l_new_$i.json 2>/dev/null || exit $?
  CGAN3D_LIB_PATH=$OLD timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4l_old_$i.json 2>/dev/null || exit $?
done
