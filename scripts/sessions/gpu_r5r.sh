#!/bin/bash
# round 5, session r: codec GEMM with the DMA issued by half the waves (out-of-phase SIMD
# pairs, TTS_CODEC_X3P_PP=1) against the default; bits by md5; stamps split of the former
set -u
O=gpurun_out
T=${1:-r5r}
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for v in 0 1; do
    TTS_CODEC_X3P_PP=$v timeout -k 10 120 python scripts/codec_probe32.py 32 650 2>&1 | grep codes >> $O/${T}_ab_codec_pp.txt || exit $?
    echo "  (TTS_CODEC_X3P_PP=$v)" >> $O/${T}_ab_codec_pp.txt
  done
done
cat $O/${T}_ab_codec_pp.txt
TTS_CODEC_X3P_PP=1 TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so TTS_CODEC_STAMPS=1 timeout -k 10 120 \
  python scripts/codec_probe32.py 32 650 2>&1 | grep -v amdgpu.ids > $O/${T}_codec_stamps_pp.txt
rc=$?
cat $O/${T}_codec_stamps_pp.txt
exit $rc
