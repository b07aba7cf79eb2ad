#!/bin/bash
# round 6: two flagged units in flight in the screen's exact recompute at K 4096 (TTS-1-Max;
# the second unit's tiles in AGPRs) vs one (-DTTS_SCR_DB32=0); the head parity tests
set -u
O=gpurun_out
T=${1:-r6ak}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_head_screen.py -v -rf --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -6 $O/${T}_tests.log; fatal $rc tests
L=tts-max_amd/tts_amd
AB_ARCH=tts1-max AB_V0=$L/libtts_db0.so AB_V1=$L/libtts_mi355x.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_db32_max8.txt 2>&1; rc=$?
cat $O/${T}_ab_db32_max8.txt; fatal $rc db32
echo done
