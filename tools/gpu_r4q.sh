# The critic's bias sums + first-layer weight grad handed to the second side stream after the
# gradient-penalty forward-mode chain instead of before it (CGAN3D_TUNE=102=1): step tests under the
# knob, then interleaved steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
CGAN3D_TUNE=102=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4q_step.log 2>&1 || { echo "step rc=$?" >> gpurun_out/r4q_step.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4q_def_$i.json 2>/dev/null || exit $?
  CGAN3D_TUNE=102=1 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4q_late_$i.json 2>/dev/null || exit $?
done
