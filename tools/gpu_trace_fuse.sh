# Kernel traces of the default bench with the fused ResNet-chain BatchNorm on and off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/tf_on $R/gpurun_out/tf_off
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tf_on -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/tf_on.json 2> $R/gpurun_out/tf_on.err || exit $?
CGAN3D_NO_BN_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tf_off -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/tf_off.json 2> $R/gpurun_out/tf_off.err
