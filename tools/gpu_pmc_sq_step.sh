# SQ issue / wait counters of the step's main kernels (KERNEL regex) inside eager bench steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_sq_step
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "${KERNEL:-conv_k3_kernel|k7s_w2n|conv_s2t|k7m_n2w|wgrad_k3_kernel|wgrad_s2_kernel}" --output-format csv -d $R/gpurun_out/pmc_sq_step -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_sq_step.log 2>&1
