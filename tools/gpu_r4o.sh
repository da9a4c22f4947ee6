# Hardware queues per process: 16 against the package default 8, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4o_q8_$i.json 2>/dev/null || exit $?
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4o_q16_$i.json 2>/dev/null || exit $?
done
