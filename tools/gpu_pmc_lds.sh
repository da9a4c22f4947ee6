# LDS bank conflicts / busy of a kernel (KERNEL regex) under tools/bench_ops.py CASE
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_lds
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$KERNEL" --output-format csv -d $R/gpurun_out/pmc_lds -o run -- python3 $R/tools/bench_ops.py --case $CASE --reps 5 > $R/gpurun_out/pmc_lds.log 2>&1
