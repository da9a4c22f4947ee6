# The critic first-layer weight grad on fewer, longer blocks (tuning key 18 = 3: 8 tiles per block),
# interleaved with the default (6 tiles per block, 256 blocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "c1 or critic or conv3d" --timeout 120 --timeout-method thread > gpurun_out/r4r_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4r_ops.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4r_def_$i.json 2>/dev/null || exit $?
  CGAN3D_TUNE=18=3 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4r_t8_$i.json 2>/dev/null || exit $?
done
