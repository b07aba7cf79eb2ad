#!/bin/bash
# round 5, session n: what the RMSNorm prologue costs now (batched LDS reads): TTS-1-Max 8-row
# and TTS-1 8-row stamps and the no-norm bound (diagnostic build, TTS_WGEMM_DIAG=16 skips the
# norm: wrong values, timing only)
set -u
O=gpurun_out
T=${1:-r5n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 || exit $?
cat $O/${T}_stamps_max8.txt
export AB_V0=0 AB_V1=16 TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_WGEMM_DIAG 8 1 > $O/${T}_ab_nonorm_max8.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/env_ab_probe.py TTS_WGEMM_DIAG 8 1 > $O/${T}_ab_nonorm_8.txt 2>&1
rc=$?
cat $O/${T}_ab_nonorm_max8.txt $O/${T}_ab_nonorm_8.txt
exit $rc
