# Round-4 bring-up of the new kernels (conv_k3m, wgrad_k3m, branch-free conv_sk, bf16 storage):
# the op tests, the step / config tests that route through them, the default bench line, and a
# kernel-trace summary of a short plan-mode bench (per-kernel averages).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k3m_ops.log 2>&1 || { echo "ops rc=$?" >> gpurun_out/k3m_ops.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -q --timeout 200 --timeout-method thread > gpurun_out/k3m_step.log 2>&1; echo "step rc=$?" >> gpurun_out/k3m_step.log
timeout -k 10 200 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/k3m_bench.json 2> gpurun_out/k3m_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/k3m_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-sub --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/k3m_prof.log 2>&1
