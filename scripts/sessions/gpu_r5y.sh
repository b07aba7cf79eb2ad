#!/bin/bash
# round 5, session y: the RMSNorm prologue's VALU cut: (1) no redundant second rounding before
# the pack (ablib/lib_rbf.so), (2) + the norm weight expanded to fp32 once per workgroup
# (in-tree); GPU suite on (2), LM A/B against session i's library and against (1) (ids md5
# must match), SIMD-tagged stamps of (2)
set -u
O=gpurun_out
T=${1:-r5y}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
export AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
AB_ARCH=tts1-max AB_V0=$PWD/ablib/lib_r5i.so timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1 || exit $?
AB_ARCH=tts1-max AB_V0=$PWD/ablib/lib_rbf.so timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8_rbf.txt 2>&1 || exit $?
AB_V0=$PWD/ablib/lib_r5i.so timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_8.txt 2>&1 || exit $?
AB_V0=$PWD/ablib/lib_r5i.so timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 1 1 > $O/${T}_ab_1.txt 2>&1 || exit $?
cat $O/${T}_ab_max8.txt $O/${T}_ab_max8_rbf.txt $O/${T}_ab_8.txt $O/${T}_ab_1.txt
TTS_WGEMM_DIAG=64 timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max 2>&1 | grep -v amdgpu.ids > $O/${T}_stamps_max8_simd.txt
rc=$?
head -8 $O/${T}_stamps_max8_simd.txt
exit $rc
