# Back-to-back A/B of two builds of the library: the in-tree build vs ab/libcgan3d_base.so
# (CGAN3D_LIB_PATH), default bench, three rounds each, interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for k in 1 2 3; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abl_new_$k.json 2> gpurun_out/abl_new_$k.err || exit $?
CGAN3D_LIB_PATH=$GRAFT_REPO_ROOT/ab/libcgan3d_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abl_base_$k.json 2> gpurun_out/abl_base_$k.err || exit $?
done
