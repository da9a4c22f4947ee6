# Back-to-back A/B of the in-tree library against builds in ab/ (ab/libcgan3d_<name>.so for each
# name in $AB_LIBS, via CGAN3D_LIB_PATH): two interleaved rounds, default bench (+ $AB_ARGS).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abn_def_$k.json 2> gpurun_out/abn_def_$k.err || exit $?
for v in $AB_LIBS; do
CGAN3D_LIB_PATH=$GRAFT_REPO_ROOT/ab/libcgan3d_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} \
  > gpurun_out/abn_${v}_$k.json 2> gpurun_out/abn_${v}_$k.err || exit $?
done
done
