#!/bin/bash
# round 5, session o: RMSNorm scaling on the A fragments (statistic-only prologue) for the
# LDS-DMA norm launches outside the fused QKV + attention launch (gate/up, lm_head at 2..16
# rows, TTS-1-Max QKV); GPU suite, LM A/B against session i's library (ids md5 must match)
set -u
O=gpurun_out
T=${1:-r5o}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
export AB_V0=$PWD/ablib/lib_r5i.so AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_8.txt 2>&1 || exit $?
cat $O/${T}_ab_8.txt
AB_ARCH=tts1-max timeout -k 10 500 python scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_max8.txt
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 16 1 > $O/${T}_ab_16.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 1 1 > $O/${T}_ab_1.txt 2>&1
rc=$?
cat $O/${T}_ab_16.txt $O/${T}_ab_1.txt
exit $rc
