#!/bin/bash
# round 6: the screened lm_head, fp32 prologue sums + two flagged units in flight in the recompute:
# same-bits switches, A/B of the wait for every workgroup's bounds (TTS_HEAD_SCREEN_WAIT) at 1
# and 8 rows, A/B of the screen vs the full lm_head at 1 / 8 / 16 rows and TTS-1-Max 8 rows
set -u
O=gpurun_out
T=${1:-r6x}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_head_screen.py tests/test_gpu_switches.py -k "head or HEAD" -v -rf --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -12 $O/${T}_tests.log; fatal $rc tests
for r in 1; do
  timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN_WAIT $r 2 > $O/${T}_ab_head_wait_$r.txt 2>&1; rc=$?
  cat $O/${T}_ab_head_wait_$r.txt; fatal $rc abw$r
done
for r in 1 8 16; do
  timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN $r 2 > $O/${T}_ab_head_screen_$r.txt 2>&1; rc=$?
  cat $O/${T}_ab_head_screen_$r.txt; fatal $rc ab$r
done
AB_ARCH=tts1-max timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN 8 2 > $O/${T}_ab_head_screen_max8.txt 2>&1; rc=$?
cat $O/${T}_ab_head_screen_max8.txt; fatal $rc abmax8
echo done
