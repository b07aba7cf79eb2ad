#!/bin/bash
# Run one gpurun call, retrying ONLY when no box/slot was free (exit 3: nothing ran, nothing
# charged), up to 20 times, 90 s apart.  Any other exit code (the command ran) is final.
# usage: scripts/gpurun_retry.sh OUTFILE TIMEOUT SCRIPT
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1; rc=$?
  echo "exit $rc (attempt $i)" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
