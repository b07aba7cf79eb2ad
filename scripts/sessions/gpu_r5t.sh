#!/bin/bash
# round 5, session t: per-wave RMSNorm-end stamps (stamps build, TTS_WGEMM_DIAG=64: the "waves
# streamed" columns then hold each wave's norm end), TTS-1-Max 8 rows
set -u
O=gpurun_out
T=${1:-r5t}
mkdir -p $O
export TMPDIR=/tmp
TTS_WGEMM_DIAG=64 timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_max8_normwaves.txt
rc=$?
head -16 $O/${T}_stamps_max8_normwaves.txt
exit $rc
