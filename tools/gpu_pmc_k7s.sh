# SQ issue / wait counters and LDS bank conflicts of the streamed-plane last conv (tools/k7s_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_k7s_a $R/gpurun_out/pmc_k7s_b
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex k7s_w2n --output-format csv -d $R/gpurun_out/pmc_k7s_a -o run -- python3 $R/tools/k7s_probe.py > $R/gpurun_out/pmc_k7s_a.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-include-regex k7s_w2n --output-format csv -d $R/gpurun_out/pmc_k7s_b -o run -- python3 $R/tools/k7s_probe.py > $R/gpurun_out/pmc_k7s_b.log 2>&1
