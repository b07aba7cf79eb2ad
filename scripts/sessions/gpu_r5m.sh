#!/bin/bash
# round 5, session m: the GEMM kernel's single/multi-unit forms chosen before any load is in
# flight (no ring copies + vmcnt(0) before the first MFMA); GPU suite, LM A/B against session
# i's library at 1, 8, 32 rows and the TTS-1-Max 8-row shard
set -u
O=gpurun_out
T=${1:-r5m}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
export AB_V0=$PWD/ablib/lib_r5i.so AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 1 2 > $O/${T}_ab_1.txt 2>&1 || exit $?
cat $O/${T}_ab_1.txt
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_8.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 32 1 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1
rc=$?
cat $O/${T}_ab_8.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
exit $rc
