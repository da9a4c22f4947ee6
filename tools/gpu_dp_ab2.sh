# one-rank DP: bucketed (default) vs one generator all-reduce on the main stream, vs no DP
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
for i in 1 2; do
MASTER_PORT=2961$i CGAN3D_FORCE_DP=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpb_bucket$i.json 2> gpurun_out/dpb.err || exit $?
MASTER_PORT=2962$i CGAN3D_FORCE_DP=1 CGAN3D_G_BUCKET_BYTES=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpb_one$i.json 2>> gpurun_out/dpb.err || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/dpb_none$i.json 2>> gpurun_out/dpb.err || exit $?
done
