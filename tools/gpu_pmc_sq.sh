# issue / wait breakdown of a kernel (KERNEL regex) under tools/bench_ops.py CASE
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_sq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "$KERNEL" --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python3 $R/tools/bench_ops.py --case $CASE --reps 5 > $R/gpurun_out/pmc_sq.log 2>&1
