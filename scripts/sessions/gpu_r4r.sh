#!/bin/bash
# round-4: a four-stage ring for the 2..16-row gate/up launch (TTS_RING4) vs two stages
set -u
O=gpurun_out
T=${1:-r4r}
mkdir -p $O
export TMPDIR=/tmp
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_RING4 8 2 > $O/${T}_ab_ring4_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_RING4 8 1 > $O/${T}_ab_ring4_tts1_8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_RING4 16 1 > $O/${T}_ab_ring4_tts1_16.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_RING4 2 1 > $O/${T}_ab_ring4_tts1_2.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
