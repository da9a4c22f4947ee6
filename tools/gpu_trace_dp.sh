# kernel trace of the one-rank RCCL data-parallel bench (CGAN3D_FORCE_DP=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/trace_dp
CGAN3D_FORCE_DP=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_dp -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/trace_dp.json 2> $R/gpurun_out/trace_dp.err
