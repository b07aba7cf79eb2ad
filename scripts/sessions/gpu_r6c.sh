#!/bin/bash
# r6c (library frozen as ablib/lib_r6c.so): RMSNorm once per row by the producing launches
# (TTS_NORM_ONCE 0/1 at TTS-1 4 / 8 / 16 rows and TTS-1-Max 8 rows), the 17..32-row fused
# launch with it (TTS_FATTN_ROWS 16/32), then the whole GPU suite.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp TTS_LIB_PATH=ablib/lib_r6c.so
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 8 3 > $OUT/r6c_normonce_8.txt 2>&1; rc=$?; cat $OUT/r6c_normonce_8.txt; fatal $rc n8
AB_ARCH=tts1-max timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 8 2 > $OUT/r6c_normonce_max8.txt 2>&1; rc=$?; cat $OUT/r6c_normonce_max8.txt; fatal $rc nmax8
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 16 2 > $OUT/r6c_normonce_16.txt 2>&1; rc=$?; cat $OUT/r6c_normonce_16.txt; fatal $rc n16
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_NORM_ONCE 4 2 > $OUT/r6c_normonce_4.txt 2>&1; rc=$?; cat $OUT/r6c_normonce_4.txt; fatal $rc n4
AB_V0=16 AB_V1=32 timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_FATTN_ROWS 32 2 > $OUT/r6c_frows32.txt 2>&1; rc=$?; cat $OUT/r6c_frows32.txt; fatal $rc f32
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/r6c_tests.log 2>&1; rc=$?; tail -8 $OUT/r6c_tests.log; fatal $rc tests
