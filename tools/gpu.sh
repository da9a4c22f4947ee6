# One parameterised GPU recipe script (replaces the per-experiment tools/gpu_r*.sh of rounds 1-4,
# which remain in git history).  Run on the box as
#     gpurun -- 'bash tools/gpu.sh <recipe> [<recipe> ...]'
# Recipes (each step under its own time limit; a timeout / kill / crash ends the script):
#   suite            pytest -m gpu (per-test durations) -> gpurun_out/gpu_tests.log
#   steptests        the ops + step + configs tests only  -> gpurun_out/step_tests.log
#   bench            default bench line (BENCH_ARGS)      -> gpurun_out/bench.json
#   ab               VARIANTS=';'-separated env lists ("-" = defaults) benched back to back, ROUNDS
#                    times (default 2), e.g. VARIANTS="-;CGAN3D_LIB_PATH=ab/libcgan3d_base.so"
#                    -> gpurun_out/ab.txt (ms_per_step per run)
#   trace            plan-mode kernel trace of the bench  -> gpurun_out/trace/ (+ TAG)
#   pmc-traffic      FETCH_SIZE / WRITE_SIZE passes over KERNEL (regex) in eager bench steps
#   pmc-sq           SQ issue / wait counters over KERNEL
#   pmc-mfma         MFMA busy cycles + GRBM active over KERNEL
#   configs          bench lines of the other single-GPU BASELINE configs and paths
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${GPU_OUT:-$R/gpurun_out}
mkdir -p $O
export TMPDIR=/tmp
KERNEL=${KERNEL:-.}
EAGER="--steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager ${BENCH_ARGS}"
chk() { local rc=$1; if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; }
for recipe in "$@"; do
  case $recipe in
    suite)
      (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=40 --timeout 300 --timeout-method thread \
        > $O/gpu_tests.log 2>&1); rc=$?; echo "tests rc=$rc" >> $O/gpu_tests.log; chk $rc ;;
    steptests)
      (cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_step.py tests/test_gpu_configs.py \
        -m gpu -q --timeout 300 --timeout-method thread > $O/step_tests.log 2>&1); rc=$?
      echo "tests rc=$rc" >> $O/step_tests.log; chk $rc ;;
    bench)
      (cd $R && timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err); chk $? ;;
    ab)
      IFS=';' read -ra VS <<< "${VARIANTS:--}"
      for k in $(seq 1 ${ROUNDS:-2}); do
        i=0
        for v in "${VS[@]}"; do
          [ "$v" = "-" ] && v=""
          (cd $R && env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-sub ${BENCH_ARGS} \
            > $O/ab_${k}_$i.json 2> $O/ab_${k}_$i.err); chk $?
          echo "$k $i [$v] $(python3 -c "import json; d=json.load(open('$O/ab_${k}_$i.json')); print(d['ms_per_step'], d['step_ms']['median'])")" >> $O/ab.txt
          i=$((i+1))
        done
      done ;;
    trace)
      rm -rf $O/trace${TAG}
      (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace${TAG} -o run -- \
        python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub ${BENCH_ARGS} > $O/trace${TAG}.json \
        2> $O/trace${TAG}.err); chk $? ;;
    pmc-traffic)
      rm -rf $O/fetch${TAG} $O/write${TAG}
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KERNEL" --output-format csv \
        -d $O/fetch${TAG} -o run -- python3 $R/bench.py $EAGER > $O/fetch${TAG}.log 2>&1); chk $?
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KERNEL" --output-format csv \
        -d $O/write${TAG} -o run -- python3 $R/bench.py $EAGER > $O/write${TAG}.log 2>&1); chk $? ;;
    pmc-sq)
      rm -rf $O/sq${TAG}
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "$KERNEL" --output-format csv \
        -d $O/sq${TAG} -o run -- python3 $R/bench.py $EAGER > $O/sq${TAG}.log 2>&1); chk $? ;;
    pmc-mfma)
      rm -rf $O/mfma${TAG}
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA \
        GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$KERNEL" --output-format csv -d $O/mfma${TAG} -o run -- \
        python3 $R/bench.py $EAGER > $O/mfma${TAG}.log 2>&1); chk $? ;;
    configs)
      (cd $R && timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-sub --size 32 --batch 1 > $O/b32_bf16.json 2> $O/b32.err); chk $?
      (cd $R && timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-sub --via-trainer > $O/b_trainer.json 2> $O/b_trainer.err); chk $?
      (cd $R && CGAN3D_FORCE_DP=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-sub \
        > $O/b_dp1.json 2> $O/b_dp1.err); chk $? ;;
    *) echo "unknown recipe $recipe"; exit 2 ;;
  esac
done
echo "gpu.sh done: $*"
