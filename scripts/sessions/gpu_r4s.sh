#!/bin/bash
# round-4: o_proj fused behind the 2..16-row attention of the QKV launch (TTS_FUSED_OPROJ_ROWS)
set -u
O=gpurun_out
T=${1:-r4s}
mkdir -p $O
export TMPDIR=/tmp
AB_ARCH=tts1-max timeout -k 10 500 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 8 2 > $O/${T}_ab_foproj_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 8 2 > $O/${T}_ab_foproj_tts1_8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 16 1 > $O/${T}_ab_foproj_tts1_16.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 2 1 > $O/${T}_ab_foproj_tts1_2.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
