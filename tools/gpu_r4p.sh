# Host-schedule knobs after the round-4 kernel changes: ResNet weight-grad hand-off group (key 100,
# default 2) and the main-stream weight-grad tail (key 101, default 2), interleaved with the default.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for t in 100=1 100=4 101=1 101=3; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4p_def_$t.json 2>/dev/null || exit $?
  CGAN3D_TUNE=$t timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4p_$t.json 2>/dev/null || exit $?
done
