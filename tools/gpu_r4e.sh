# conv_k3m epilogue variants: accumulator replicas 16 / 64, no statistics, no residual.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_fwd_k3m_r64 res_fwd_k3m_nostat res_fwd_k3m_plain res_dgrad_k3m res_dgrad_k3m_r64 > gpurun_out/r4e_probe.txt 2>&1
