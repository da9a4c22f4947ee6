# Same-box A/B of the current library against the r4i-verified build (contrast-gan-3d_amd/ab,
# CGAN3D_LIB_PATH), interleaved; then the halo-ring knob (key 21) and single-kernel probes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
OLD=$R/contrast-gan-3d_amd/ab/libcgan3d_e4d2.so
for i in 1 2 3; do
  CGAN3D_LIB_PATH=$OLD timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4k_old_$i.json 2>/dev/null || exit $?
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4k_new_$i.json 2>/dev/null || exit $?
done
CGAN3D_TUNE=21=0 timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4k_ring.json 2>/dev/null || exit $?
timeout -k 10 200 python -u tools/bench_ops.py --case up0_fwd down1_fwd crit_first crit_m0 crit_m1 crit_m2 > gpurun_out/r4k_probe.txt 2>&1 || exit $?
CGAN3D_LIB_PATH=$OLD timeout -k 10 200 python -u tools/bench_ops.py --case up0_fwd down1_fwd crit_first crit_m0 crit_m1 crit_m2 >> gpurun_out/r4k_probe.txt 2>&1 || exit $?
