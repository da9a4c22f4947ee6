# A/B: plain single-GPU bench vs the data-parallel path over a one-rank RCCL group (CGAN3D_FORCE_DP=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  timeout -k 10 120 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep metric > $R/gpurun_out/dp_a$rep.json || exit $?
  CGAN3D_FORCE_DP=1 timeout -k 10 120 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>$R/gpurun_out/dp_b.err | grep metric > $R/gpurun_out/dp_b$rep.json || exit $?
done
