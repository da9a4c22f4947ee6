# Which of the post-r4i changes costs the ~5 us: interleaved steps of the r4i build (e4d2), the
# current build with the old BatchNorm passes (A), with the old critic conv.hip / conv_c1.hip (B), and
# the current build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
AB=$R/contrast-gan-3d_amd/ab
for i in 1 2; do
  for v in e4d2 A B; do
    CGAN3D_LIB_PATH=$AB/libcgan3d_$v.so timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4m_${v}_$i.json 2>/dev/null || exit $?
  done
  timeout -k 10 120 python -u bench.py --no-sub --no-cpu-baseline > gpurun_out/r4m_new_$i.json 2>/dev/null || exit $?
done
