#!/bin/bash
# usage: gpuq.sh OUTFILE TIMEOUT cmd...   — retries the gpurun client while no slot/box is free (rc 3 / transient)
out=$1; shift; to=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1; rc=$?
  if grep -q "status=transient\|rc=3\|slot(s) on this pod are busy\|backing off" $out && ! grep -q "status=ok" $out; then
    sleep 90; continue
  fi
  echo "rc=$rc" >> $out; exit $rc
done
echo "gave up" >> $out
