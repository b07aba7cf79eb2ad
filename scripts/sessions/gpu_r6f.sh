#!/bin/bash
# r6f (ablib/lib_r6f.so): the down projection K-sliced at 2..9 rows too, so its combine
# normalises each row once for the next QKV launch (TTS_SLICE_RESID_ROWS 0 vs 2)
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp TTS_LIB_PATH=ablib/lib_r6f.so
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
for rows in 8 4 2; do
  AB_V0=0 AB_V1=2 timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_SLICE_RESID_ROWS $rows 2 > $OUT/r6f_slice_$rows.txt 2>&1; rc=$?; cat $OUT/r6f_slice_$rows.txt; fatal $rc s$rows
done
