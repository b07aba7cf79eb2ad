#!/bin/bash
# round 5, session k: codec GEMM tile A/B: 256x128 two stages (default) vs 128x128 on 8 waves
# with three stages (TTS_CODEC_X3P_TILE=5), bits compared by md5; stamps split of the latter
set -u
O=gpurun_out
T=${1:-r5k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py -m gpu > $O/${T}_codec_tests.log 2>&1 || exit $?
tail -2 $O/${T}_codec_tests.log
for r in 0 1; do
  for v in d 5; do
    if [ $v = d ]; then unset TTS_CODEC_X3P_TILE; else export TTS_CODEC_X3P_TILE=$v; fi
    timeout -k 10 120 python scripts/codec_probe32.py 32 650 2>&1 | grep codes >> $O/${T}_ab_codec_tile.txt || exit $?
    echo "  (TTS_CODEC_X3P_TILE=$v)" >> $O/${T}_ab_codec_tile.txt
  done
done
unset TTS_CODEC_X3P_TILE
cat $O/${T}_ab_codec_tile.txt
TTS_CODEC_X3P_TILE=5 TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so TTS_CODEC_STAMPS=1 timeout -k 10 120 \
  python scripts/codec_probe32.py 32 650 2>&1 | grep -v amdgpu.ids > $O/${T}_codec_stamps_tile5.txt || exit $?
cat $O/${T}_codec_stamps_tile5.txt
