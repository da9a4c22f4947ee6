# Launch-shape sweep of the ResNet / stride-2 weight-grad grids (cgan3d_set_tuning keys 9, 10) against
# the default, interleaved on one box; one bench line per setting under gpurun_out/tune_*.json.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in def 9=20 9=40 def 9=56 10=96 def 10=192 9=40,10=192 def; do
  if [ "$cfg" = def ]; then
    timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/tune_$cfg.$RANDOM.json 2>/dev/null || exit $?
  else
    CGAN3D_TUNE=$cfg timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/tune_$cfg.json 2>/dev/null || exit $?
  fi
done
