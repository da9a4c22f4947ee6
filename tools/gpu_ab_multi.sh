# Bench under several env settings, back to back on one box (VARIANTS: ';'-separated env lists,
# "-" = defaults), e.g. VARIANTS="-;CGAN3D_DEBUG=keep_fp32;-;CGAN3D_DEBUG=keep_fp32"
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:--}"
i=0
for v in "${VS[@]}"; do
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/abm_$i.json 2> gpurun_out/abm_$i.err || exit $?
  echo "$i [$v] $(python -c "import json; d=json.load(open('gpurun_out/abm_$i.json')); print(d['ms_per_step'])")" >> gpurun_out/abm.txt
  i=$((i+1))
done
