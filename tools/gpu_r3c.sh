# round 3 evidence: the validate test, PMC traffic (conv_k3), SQ counters of the step's kernels,
# DP one-rank benches (native RCCL / torch comm), the fp32 64^3 B=4 line, a kernel trace of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py -k validate_at -q -x --durations=5 --timeout 300 --timeout-method thread > gpurun_out/val.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --precision f32 > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || exit $?
CGAN3D_FORCE_DP=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dp1.json 2> gpurun_out/bench_dp1.err || exit $?
CGAN3D_FORCE_DP=1 CGAN3D_TORCH_COMM=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_dp1_torch.json 2> gpurun_out/bench_dp1_torch.err || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write $R/gpurun_out/pmc_sq_step $R/gpurun_out/trace_main
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "conv_k3_kernel|k7s_w2n|conv_s2t|conv_s2f|k7m_n2w|wgrad_k3_kernel|wgrad_s2|conv_sk|bn_" --output-format csv -d $R/gpurun_out/pmc_sq_step -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/pmc_sq_step.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_main -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/trace_main.json 2> $R/gpurun_out/trace_main.err
