# A/B of an environment switch on the default bench, back to back on one box:
#   AB_ENV="CGAN3D_BN_INLAUNCH=0" gpurun -- bash tools/gpu_ab_env.sh   -> gpurun_out/ab_{a,b}{1,2}.json
set -o pipefail
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  timeout -k 10 120 python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline $BENCH_ARGS > $R/gpurun_out/ab_a$rep.json 2> $R/gpurun_out/ab_a$rep.err || exit $?
  timeout -k 10 120 env $AB_ENV python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline $BENCH_ARGS > $R/gpurun_out/ab_b$rep.json 2> $R/gpurun_out/ab_b$rep.err || exit $?
done
