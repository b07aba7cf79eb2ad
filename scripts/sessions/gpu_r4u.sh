#!/bin/bash
# round-4: fused 2..16-row o_proj with its granule polls batched over 4 rows: stamps, A/B, bits
set -u
O=gpurun_out
T=${1:-r4u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 8 > $O/${T}_stamps_tts1_8.txt 2>&1 && \
AB_ARCH=tts1-max timeout -k 10 500 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 8 1 > $O/${T}_ab_foproj_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 8 1 > $O/${T}_ab_foproj_tts1_8.txt 2>&1 && \
timeout -k 10 300 python scripts/env_ab_probe.py TTS_FUSED_OPROJ_ROWS 16 1 > $O/${T}_ab_foproj_tts1_16.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_launch.py > $O/${T}_tests.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
