#!/bin/bash
# r6e: decode attention with interleaved position blocks at head dim 64 (ablib/lib_r6e.so)
# against r6d's library (contiguous blocks), TTS_NORM_ONCE=3 in both (same norm form); then
# TTS_NORM_ONCE 0 vs 3 (the K-sliced down's combine normalising at 10..16 rows) on r6e; then
# the LM parity tests on r6e.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp TTS_NORM_ONCE=3
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
ab() {  # rows rounds [arch]
  AB_ARCH=${3:-tts1} AB_V0=ablib/lib_r6d.so AB_V1=ablib/lib_r6e.so timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_LIB_PATH $1 $2 > $OUT/r6e_ilv_${3:-tts1}_$1.txt 2>&1; local rc=$?; cat $OUT/r6e_ilv_${3:-tts1}_$1.txt; fatal $rc ilv$1
}
ab 1 3 && ab 8 2 && ab 32 2 && ab 8 2 tts1-max
export TTS_LIB_PATH=ablib/lib_r6e.so
for rows in 16 12; do
  AB_V0=0 AB_V1=3 timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_NORM_ONCE $rows 2 > $OUT/r6e_normonce3_$rows.txt 2>&1; rc=$?; cat $OUT/r6e_normonce3_$rows.txt; fatal $rc n$rows
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "lm or chain or fused or long or switch or attention or stream" > $OUT/r6e_tests.log 2>&1; rc=$?; tail -5 $OUT/r6e_tests.log; fatal $rc tests
