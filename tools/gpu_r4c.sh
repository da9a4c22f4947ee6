# Round 4: host-schedule sweep (CGAN3D_TUNE 100 = weight-grad hand-off group, 101 = weight grads kept
# on the main stream at the end of the backward), interleaved with the default, and the 128^3 B=1
# fp32 configuration (BASELINE configs[2]) under a kernel trace (per-kernel GB/s of its BatchNorm /
# elementwise passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for cfg in def 100=3 101=1 def 100=4 101=3 100=1 def; do
  if [ $cfg = def ]; then T=""; else T=$cfg; fi
  CGAN3D_TUNE=$T timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4c_$cfg.$RANDOM.json 2>/dev/null || exit $?
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r4c_b128
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4c_b128 -o run -- python3 $R/bench.py --size 128 --batch 1 --precision f32 --steps 10 --warmup 2 --no-sub --no-cpu-baseline > $R/gpurun_out/r4c_b128.json 2> $R/gpurun_out/r4c_b128.err
cd $R && timeout -k 10 200 python -u tools/bench_ops.py --case res_fwd_k3m res_dgrad_k3m res_wgrad --tune 17=0,1,2,3,4,8,12,7,15 > gpurun_out/k3m_probe.txt 2>&1
