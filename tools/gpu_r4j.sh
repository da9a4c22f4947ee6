# k7 weight-grad grid A/B (tuning key 20), interleaved with the default, then a plan-mode kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in 128 256; do
  CGAN3D_TUNE=20=$v timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4j_bench_k7wg$v.json 2>/dev/null || exit $?
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4j_bench_def$v.json 2>/dev/null || exit $?
done
timeout -k 10 200 python -u tools/bench_ops.py --case k7_last_wgrad k7_first_wgrad --tune 20=512,256,128 > gpurun_out/r4j_probe.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r4j_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4j_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $R/gpurun_out/r4j_trace.json 2> $R/gpurun_out/r4j_trace.err
