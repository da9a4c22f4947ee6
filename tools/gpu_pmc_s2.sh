# SQ issue / wait counters and L2 / HBM traffic of the stride-2 kernels under tools/s2_probe.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${KERNEL:-conv_s2}
rm -rf $R/gpurun_out/pmc_s2_a $R/gpurun_out/pmc_s2_b $R/gpurun_out/pmc_s2_c
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVES --kernel-include-regex $K --output-format csv -d $R/gpurun_out/pmc_s2_a -o run -- python3 $R/tools/s2_probe.py > $R/gpurun_out/pmc_s2_a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d $R/gpurun_out/pmc_s2_b -o run -- python3 $R/tools/s2_probe.py > $R/gpurun_out/pmc_s2_b.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex $K --output-format csv -d $R/gpurun_out/pmc_s2_c -o run -- python3 $R/tools/s2_probe.py > $R/gpurun_out/pmc_s2_c.log 2>&1
