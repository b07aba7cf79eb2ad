#!/bin/bash
# round 5, session x: which waves finish the RMSNorm prologue late — norm end per wave with its
# SIMD (stamps build, TTS_WGEMM_DIAG=64), TTS-1-Max 8 rows and TTS-1 8 rows
set -u
O=gpurun_out
T=${1:-r5x}
mkdir -p $O
export TMPDIR=/tmp
TTS_WGEMM_DIAG=64 timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_max8_simd.txt || exit $?
TTS_WGEMM_DIAG=64 timeout -k 10 300 python scripts/stamp_probe.py 452 8 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_8_simd.txt
rc=$?
grep -B6 -A3 "by SIMD" $O/${T}_stamps_max8_simd.txt | head -40
grep -A3 "by SIMD" $O/${T}_stamps_8_simd.txt | head -20
exit $rc
