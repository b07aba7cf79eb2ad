#!/bin/bash
# round 5, session c: GPU suite on the buffer-load weight stream + the planes codec GEMM
# (gemm_x3p), codec A/B (TTS_CODEC_X3P 0/1: time + waveform md5), LM A/B vs the r5a library
set -u
O=gpurun_out
T=${1:-r5c}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for r in 1 2; do
  for v in 0 1; do
    TTS_CODEC_X3P=$v timeout -k 10 120 python scripts/codec_probe32.py 32 650 >> $O/${T}_ab_codec.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P=$v)" >> $O/${T}_ab_codec.txt
    TTS_CODEC_X3P=$v timeout -k 10 120 python scripts/codec_probe32.py 1 650 >> $O/${T}_ab_codec.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P=$v)" >> $O/${T}_ab_codec.txt
  done
done
cat $O/${T}_ab_codec.txt
export AB_V0=$PWD/ablib/lib_r5a.so AB_V1=$PWD/ablib/lib_cur.so
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 1 2 > $O/${T}_ab_1.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 32 2 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 600 python scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_max8.txt 2>&1
rc=$?
cat $O/${T}_ab_1.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
exit $rc
