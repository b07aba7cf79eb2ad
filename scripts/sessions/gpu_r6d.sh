#!/bin/bash
# r6d (library frozen as ablib/lib_r6d.so): TTS_NORM_ONCE modes — 0 (prologue norms) vs 2
# (norm workgroups in the fused QKV + attention + o_proj launch, the K-sliced down's combine
# normalising; no norm workgroups on the down launch) at TTS-1 4 / 8 / 16 rows and TTS-1-Max 8.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp TTS_LIB_PATH=ablib/lib_r6d.so
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
for rows in 8 16 4; do
  AB_V0=0 AB_V1=2 timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_NORM_ONCE $rows 2 > $OUT/r6d_normonce_$rows.txt 2>&1; rc=$?; cat $OUT/r6d_normonce_$rows.txt; fatal $rc n$rows
done
AB_ARCH=tts1-max AB_V0=0 AB_V1=2 timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 8 2 > $OUT/r6d_normonce_max8.txt 2>&1; rc=$?; cat $OUT/r6d_normonce_max8.txt; fatal $rc nmax8
AB_V0=0 AB_V1=2 timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 12 2 > $OUT/r6d_normonce_12.txt 2>&1; rc=$?; cat $OUT/r6d_normonce_12.txt; fatal $rc n12
