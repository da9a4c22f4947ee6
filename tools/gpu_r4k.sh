# Single-kernel probes and interleaved A/B of the round-4 knobs (keys 20, 21).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_ops.py --case up0_fwd down1_fwd --tune 21=1,0,2 > gpurun_out/r4k_probe.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case crit_first crit_m0 crit_m1 crit_m2 >> gpurun_out/r4k_probe.txt 2>&1 || exit $?
for t in 21=0 20=256; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4k_bench_def_$t.json 2>/dev/null || exit $?
  CGAN3D_TUNE=$t timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4k_bench_$t.json 2>/dev/null || exit $?
done
