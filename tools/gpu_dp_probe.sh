# which part of the one-rank DP setup slows the step: the process group alone, a second (own)
# communicator, the DP step on torch's communicator (default) and on an own one
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
MASTER_PORT=29581 CGAN3D_FORCE_DP=native timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpp_native.json 2> gpurun_out/dpp_native.err || exit $?
MASTER_PORT=29582 CGAN3D_FORCE_DP=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpp_1.json 2> gpurun_out/dpp_1.err || exit $?
MASTER_PORT=29583 CGAN3D_FORCE_DP=1 CGAN3D_COMM=own timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpp_own.json 2> gpurun_out/dpp_own.err || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpp_none.json 2> gpurun_out/dpp_none.err || exit $?
MASTER_PORT=29584 CGAN3D_FORCE_DP=1 timeout -k 10 300 python -u tools/dist_nccl1_check.py > gpurun_out/dn1.log 2>&1
