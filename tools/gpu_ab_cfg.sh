# A/B of an environment switch with the bf16 parity subset first: default vs $AB_ENV, two rounds each.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_step.py \
  tests/test_gpu_trainer.py tests/test_gpu_dist.py -k "${AB_K:-(bf16 and 64) or plan_replay or accumulators or fixture or trainer or dist or rank}" \
  > gpurun_out/abc_tests.log 2>&1 || exit $?
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abc_def_$k.json 2> gpurun_out/abc_def_$k.err || exit $?
env $AB_ENV timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abc_alt_$k.json 2> gpurun_out/abc_alt_$k.err || exit $?
done
