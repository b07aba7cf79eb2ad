#!/bin/bash
set -u
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_BALANCE 8 1 > $O/r4q_ab_balance_max8.txt 2>&1 && \
AB_ARCH=tts1-max AB_V0=0 AB_V1=16 timeout -k 10 400 python scripts/env_ab_probe.py TTS_FATTN_ROWS 8 1 > $O/r4q_ab_fattn_max8.txt 2>&1 && \
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_AGR 8 1 > $O/r4q_ab_agr_max8.txt 2>&1
echo "rc=$?"
