#!/bin/bash
# gpurun, retried only while no box or slot is free (exit 3, or a transient infrastructure status):
# nothing ran then and nothing was charged.  Any other outcome (pass, failure, timeout) ends it.
# usage: tools/gpu_retry.sh OUTFILE TRIES gpurun-args...
out=$1; tries=$2; shift 2
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then
    sleep 120
    continue
  fi
  echo "rc=$rc" >> "$out"
  exit $rc
done
echo "gave up after $tries tries" >> "$out"
