# k7 weight-grad grid (tuning key 20, default 512 blocks) against the default, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for t in 20=256 20=128 20=1024; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4n_def_$t.json 2>/dev/null || exit $?
  CGAN3D_TUNE=$t timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4n_$t.json 2>/dev/null || exit $?
done
