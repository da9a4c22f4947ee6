# one-rank DP (RCCL) bench A/B: stream / queue settings, then a kernel trace of the native path
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CGAN3D_FORCE_DP=1 MASTER_ADDR=127.0.0.1
MASTER_PORT=29571 CGAN3D_CRITIC_W0_SIDE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dp_noside.json 2> gpurun_out/dp_ab.err || exit $?
MASTER_PORT=29572 GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dp_q16.json 2>> gpurun_out/dp_ab.err || exit $?
MASTER_PORT=29573 GPU_MAX_HW_QUEUES=16 CGAN3D_CRITIC_W0_SIDE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dp_q16_noside.json 2>> gpurun_out/dp_ab.err || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/trace_dp
MASTER_PORT=29574 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_dp -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/trace_dp.json 2> $R/gpurun_out/trace_dp.err
