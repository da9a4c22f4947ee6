# bench lines of the other single-GPU BASELINE configs, the Trainer path and the one-rank RCCL path
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --no-cpu-baseline --size 128 --batch 1 --precision f32 --steps 10 --warmup 3 > gpurun_out/b128_f32.json 2> gpurun_out/b128_f32.err || exit $?
timeout -k 10 240 python -u bench.py --no-cpu-baseline --size 128 --batch 2 --steps 10 --warmup 3 > gpurun_out/b128_bf16.json 2> gpurun_out/b128_bf16.err || exit $?
timeout -k 10 240 python -u bench.py --no-cpu-baseline --size 32 --batch 1 > gpurun_out/b32_bf16.json 2> gpurun_out/b32_bf16.err || exit $?
timeout -k 10 240 python -u bench.py --no-cpu-baseline --via-trainer > gpurun_out/b_trainer.json 2> gpurun_out/b_trainer.err || exit $?
CGAN3D_FORCE_DP=1 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/b_dp1.json 2> gpurun_out/b_dp1.err
