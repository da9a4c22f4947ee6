# Round-4 final evidence, part A: the whole GPU suite (per-test durations), the default bench line
# (with its f32 / b128 sub-lines and the CPU baseline), the plan host-issue time.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=40 --timeout 240 --timeout-method thread > gpurun_out/fin_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/fin_gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || exit $?
timeout -k 10 120 python -u tools/plan_host_time.py > gpurun_out/fin_host.txt 2>&1 || exit $?
exit $rc
