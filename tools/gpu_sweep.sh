# tuning sweep (SWEEP="key=v ..."): step time under plans and the ResNet conv launch time per value
cd $GRAFT_REPO_ROOT
for t in $SWEEP; do
  echo "== $t"; CGAN3D_TUNE="$t" timeout -k 10 100 python -u tools/host_time.py 2>&1 | grep plan || exit 1
  CGAN3D_TUNE="$t" timeout -k 10 100 python -u tools/bench_ops.py --case res_fwd 2>&1 | grep res_fwd || exit 1
done > gpurun_out/sweep.log
