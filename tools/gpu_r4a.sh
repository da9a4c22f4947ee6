# Round 4: re-check the A/B step tests and the teacher-forced layer test after their fixes, then SQ
# counters (issue / wait / instruction mix, LDS bank conflicts) of the step's main kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py -k "accumulators or storage or shadows or layers" -q --timeout 200 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1; echo "rc=$?" >> gpurun_out/r4a_tests.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K='conv_k3m|wgrad_k3m|conv_sk|conv_halo|k7m_n2w|conv_s2t|conv_s2f|wgrad_s2|k7m_wg|cout1_block|conv_gemm|c1_fwd|c1_dgrad'
rm -rf $R/gpurun_out/r4a_sq $R/gpurun_out/r4a_lds
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "$K" --output-format csv -d $R/gpurun_out/r4a_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/r4a_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL --kernel-include-regex "$K" --output-format csv -d $R/gpurun_out/r4a_lds -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/r4a_lds.log 2>&1
