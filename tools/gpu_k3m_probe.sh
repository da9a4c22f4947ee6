# conv_k3m phase timing: each probe bit (tuning key 17) drops one phase (results wrong, times only):
# 1 halo DMA, 2 weight DMA, 4 MFMA loop, 8 epilogue.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_dgrad_k3m res_wgrad --tune 17=0,1,2,3,4,8,12,7,15 > gpurun_out/k3m_probe.txt 2>&1
