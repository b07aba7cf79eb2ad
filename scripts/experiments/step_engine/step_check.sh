#!/bin/bash
# GPU check of the persistent one-row step: a short generate through it and through the
# per-layer launches (TTS_STEP=0), then the kernel timings.   usage: scripts/step_check.sh TAG
set -u
TAG=$1
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/step_smoke.py > $OUT/${TAG}_step_on.log 2>&1 || { tail -20 $OUT/${TAG}_step_on.log; exit 1; }
tail -3 $OUT/${TAG}_step_on.log | cut -c1-300
TTS_STEP=0 timeout -k 10 120 python -u scripts/step_smoke.py > $OUT/${TAG}_step_off.log 2>&1 || { tail -20 $OUT/${TAG}_step_off.log; exit 1; }
tail -3 $OUT/${TAG}_step_off.log | cut -c1-300

