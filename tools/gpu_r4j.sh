# Resident weight slabs in the halo kernel (key 21) and the k7 weight-grad grid (key 20): op / step
# tests, interleaved bench A/B, single-kernel probes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/r4j_ops.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4j_step.log 2>&1; echo "rc=$?" >> gpurun_out/r4j_step.log
timeout -k 10 200 python -u tools/bench_ops.py --case up0_fwd down1_fwd --tune 21=1,0,2 > gpurun_out/r4j_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case crit_first crit_m0 crit_m1 crit_m2 >> gpurun_out/r4j_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case k7_last_wgrad k7_first_wgrad --tune 20=512,256,128 >> gpurun_out/r4j_probe.txt 2>&1 || exit $?
for t in 21=0 20=256 21=2; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4j_bench_def_$t.json 2>/dev/null || exit $?
  CGAN3D_TUNE=$t timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4j_bench_$t.json 2>/dev/null || exit $?
done
