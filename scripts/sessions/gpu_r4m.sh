#!/bin/bash
# round-4: bound the LDS prologue's RMSNorm cost at 8 rows: skipped (TTS_WGEMM_DIAG=16, wrong results:
# timing only)
set -u
O=gpurun_out
T=${1:-r4m}
mkdir -p $O
export TMPDIR=/tmp
TTS_WGEMM_DIAG=16 timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8_d16.txt 2>&1 && \
AB_ARCH=tts1-max AB_V0=0 AB_V1=16 timeout -k 10 400 python scripts/env_ab_probe.py TTS_WGEMM_DIAG 8 1 > $O/${T}_ab_max8_skipnorm.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
