# Round-4 final evidence, part B: a plan-mode kernel trace of the bench, conv_k3m HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes) and SQ counters of the step's main kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 200 python3 $R/bench.py --precision f32 --no-sub --no-cpu-baseline > $R/gpurun_out/fin_bench_f32.json 2> $R/gpurun_out/fin_bench_f32.err || exit $?
rm -rf $R/gpurun_out/fin_trace $R/gpurun_out/fin_fetch $R/gpurun_out/fin_write $R/gpurun_out/fin_sq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fin_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $R/gpurun_out/fin_trace.json 2> $R/gpurun_out/fin_trace.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_k3m_kernel --output-format csv -d $R/gpurun_out/fin_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/fin_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_k3m_kernel --output-format csv -d $R/gpurun_out/fin_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/fin_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "conv_k3m|wgrad_k3m|k7s_w2n|conv_s2t|conv_s2f|k7m_|wgrad_s2|conv_sk|c1_|conv_halo|bn_" --output-format csv -d $R/gpurun_out/fin_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager > $R/gpurun_out/fin_sq.log 2>&1
