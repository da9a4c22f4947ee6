# Three-way A/B of environment settings: default, $AB_ENV, $AB_ENV2 — two rounds each, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab3_def_$k.json 2> gpurun_out/ab3_def_$k.err || exit $?
env $AB_ENV timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab3_a_$k.json 2> gpurun_out/ab3_a_$k.err || exit $?
env $AB_ENV2 timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab3_b_$k.json 2> gpurun_out/ab3_b_$k.err || exit $?
done
