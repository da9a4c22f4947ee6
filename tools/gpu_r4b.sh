# Round 4: step / config tests, the default bench line (with its sub-lines), a weight-grad chunk
# sweep (tuning key 9), conv_k3m HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) and a
# plan-mode kernel trace.  Every step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -q --timeout 200 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1; echo "rc=$?" >> gpurun_out/r4b_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || exit $?
for cfg in 9=14 9=20 9=40; do
  CGAN3D_TUNE=$cfg timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4b_tune_$cfg.json 2>/dev/null || exit $?
done
timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4b_tune_def.json 2>/dev/null || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r4b_fetch $R/gpurun_out/r4b_write $R/gpurun_out/r4b_trace
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_k3m_kernel --output-format csv -d $R/gpurun_out/r4b_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/r4b_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_k3m_kernel --output-format csv -d $R/gpurun_out/r4b_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/r4b_write.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4b_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $R/gpurun_out/r4b_trace.json 2> $R/gpurun_out/r4b_trace.err
