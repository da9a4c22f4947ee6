# kernel traces of the single-GPU step and of the one-rank DP step (plan mode)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tr_none $R/gpurun_out/tr_dp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_none -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/tr_none.json 2> $R/gpurun_out/tr_none.err || exit $?
MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 CGAN3D_FORCE_DP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_dp -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/tr_dp.json 2> $R/gpurun_out/tr_dp.err
