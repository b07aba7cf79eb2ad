#!/bin/bash
# round 5, session p: where the RMSNorm prologue's time goes (stamps build: row statistic vs
# scaled rows, wave 0), TTS-1-Max 8 rows and TTS-1 8 rows
set -u
O=gpurun_out
T=${1:-r5p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_max8.txt || exit $?
timeout -k 10 300 python scripts/stamp_probe.py 452 8 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_8.txt
rc=$?
cat $O/${T}_stamps_max8.txt $O/${T}_stamps_8.txt
exit $rc
