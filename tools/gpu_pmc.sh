# HBM traffic of the roofline kernel (conv_k3_kernel) from separate FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_write.log 2>&1
