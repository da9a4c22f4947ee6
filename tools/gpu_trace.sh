# Kernel traces of the default bench (plan mode): with the side stream (the real schedule) and with
# everything serialised on one stream (CGAN3D_DEBUG=serial: unshared kernel durations).
#   gpurun -- bash tools/gpu_trace.sh      -> gpurun_out/trace_{main,serial}/ + .json bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-trace}
rm -rf $R/gpurun_out/${TAG}_main $R/gpurun_out/${TAG}_serial
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_main -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $R/gpurun_out/${TAG}_main.json 2> $R/gpurun_out/${TAG}_main.err || exit $?
CGAN3D_DEBUG=serial timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_serial -o run -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $R/gpurun_out/${TAG}_serial.json 2> $R/gpurun_out/${TAG}_serial.err
