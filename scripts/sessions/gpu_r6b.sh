#!/bin/bash
# r6b: the 17..32-row fused QKV + attention + o_proj launch (TTS_FATTN_ROWS 16 = round 5's
# seven-launch layer vs 32 = the fused form), the gate/up norm in the prologue at 32 rows,
# the tiled V^T layout against the round-5 library (TTS_LIB_PATH A/B, TTS-1-Max 8 rows and
# TTS-1 1 / 8 rows), the K = 768 op probe, then the batched GPU tests.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
timeout -k 10 120 python -u scripts/k768_probe.py > $OUT/r6b_k768.txt 2>&1; rc=$?; cat $OUT/r6b_k768.txt | tail -8; fatal $rc k768
AB_V0=16 AB_V1=32 timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_FATTN_ROWS 32 3 > $OUT/r6b_frows32.txt 2>&1; rc=$?; cat $OUT/r6b_frows32.txt; fatal $rc frows32
AB_V0=16 AB_V1=32 timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_FATTN_ROWS 24 2 > $OUT/r6b_frows24.txt 2>&1; rc=$?; cat $OUT/r6b_frows24.txt; fatal $rc frows24
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_NORM_PROLOGUE32 32 2 > $OUT/r6b_normpro32.txt 2>&1; rc=$?; cat $OUT/r6b_normpro32.txt; fatal $rc normpro
AB_ARCH=tts1-max AB_V0=ablib/lib_base.so AB_V1=tts-max_amd/tts_amd/libtts_mi355x.so timeout -k 10 400 python -u scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $OUT/r6b_vt_max8.txt 2>&1; rc=$?; cat $OUT/r6b_vt_max8.txt; fatal $rc vtmax
AB_V0=ablib/lib_base.so AB_V1=tts-max_amd/tts_amd/libtts_mi355x.so timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_LIB_PATH 1 2 > $OUT/r6b_vt_1.txt 2>&1; rc=$?; cat $OUT/r6b_vt_1.txt; fatal $rc vt1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "batch or chain or rows or fused or switch or tts1max or long" > $OUT/r6b_tests.log 2>&1; rc=$?; tail -5 $OUT/r6b_tests.log; fatal $rc tests
