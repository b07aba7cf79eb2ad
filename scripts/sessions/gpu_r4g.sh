#!/bin/bash
# round-4 stamps: TTS-1-Max 8 rows (QKV + attention in one launch, and separate), TTS-1 8 and 32 rows
set -u
O=gpurun_out
T=${1:-r4g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 8 > $O/${T}_stamps_tts1_8.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 32 > $O/${T}_stamps_tts1_32.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 1 > $O/${T}_stamps_tts1_1.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
