# Quick A/B of an environment switch: default vs $AB_ENV (e.g. AB_ENV=CGAN3D_DEBUG=no_bn_fold), two
# rounds each, back to back on one box, plus a plan-mode kernel trace of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$AB_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step.py -k "$AB_TESTS" > gpurun_out/ab_tests.log 2>&1 || exit $?
fi
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_def_$k.json 2> gpurun_out/ab_def_$k.err || exit $?
env $AB_ENV timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_alt_$k.json 2> gpurun_out/ab_alt_$k.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/tab
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tab -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/tab.json 2> $GRAFT_REPO_ROOT/gpurun_out/tab.err
