#!/bin/bash
# round 5, session u: the RMSNorm prologue at two waves per row (16-wave launches at <= 8 rows,
# 8-wave at <= 4); GPU suite, LM A/B against session i's library (ids md5 must match), stamps
set -u
O=gpurun_out
T=${1:-r5u}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
export AB_V0=$PWD/ablib/lib_r5i.so AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
AB_ARCH=tts1-max timeout -k 10 500 python scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_max8.txt
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 4 1 > $O/${T}_ab_4.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_8.txt 2>&1 || exit $?
cat $O/${T}_ab_4.txt $O/${T}_ab_8.txt
unset AB_V0 AB_V1
TTS_WGEMM_DIAG=64 timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_max8_normwaves.txt
rc=$?
head -6 $O/${T}_stamps_max8_normwaves.txt
exit $rc
