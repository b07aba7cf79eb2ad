#!/bin/bash
# round 5, session h: GPU suite on the all-wave RMSNorm prologue + the decode attention that
# loads q|k|v and RoPE ahead of its K / V^T fragments (same bits expected); then session g's
# PMC diagnostics and bs=32 A/Bs; A/B of the new library against r5f's
set -u
O=gpurun_out
T=${1:-r5h}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for v in 0 1; do
  for b in 32 1; do
    TTS_CODEC_X3P_ILV=$v timeout -k 10 120 python scripts/codec_probe32.py $b 650 >> $O/${T}_ab_codec_ilv.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P_ILV=$v)" >> $O/${T}_ab_codec_ilv.txt
  done
done
cat $O/${T}_ab_codec_ilv.txt
export AB_V0=$PWD/ablib/lib_cur.so AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_8.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 32 1 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_8.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
unset AB_V0 AB_V1
bash scripts/sessions/gpu_r5g.sh ${T}g
