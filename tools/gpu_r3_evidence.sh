# Round-3 evidence in one GPU call: default bench line, fp32 64^3 B=4 line, plan host-issue time,
# a plan-mode kernel trace of the bench, conv_k3 HBM traffic (separate FETCH_SIZE / WRITE_SIZE
# passes) and SQ counters of the step's main kernels.  Every step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --precision f32 > gpurun_out/ev_bench_f32.json 2> gpurun_out/ev_bench_f32.err || exit $?
timeout -k 10 120 python -u tools/plan_host_time.py > gpurun_out/ev_host.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/ev_trace $R/gpurun_out/ev_fetch $R/gpurun_out/ev_write $R/gpurun_out/ev_sq
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/ev_trace.json 2> $R/gpurun_out/ev_trace.err || exit $?
[ -n "$NO_PMC" ] && exit 0
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/ev_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/ev_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex conv_k3_kernel --output-format csv -d $R/gpurun_out/ev_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/ev_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "${KERNEL:-conv_k3_kernel|k7s_w2n|conv_s2t|conv_s2f|k7m_n2w|wgrad_k3_kernel|wgrad_s2|conv_sk|c1_}" --output-format csv -d $R/gpurun_out/ev_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --mode eager > $R/gpurun_out/ev_sq.log 2>&1
