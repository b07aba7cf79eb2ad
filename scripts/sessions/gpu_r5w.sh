#!/bin/bash
# round 5, session w: the lone utterance's codec GEMM tile: the size heuristic (32x32 one-wave
# tiles for most of its GEMMs) against every tile forced, 1 x 650 and 1 x 50 codes (bits equal)
set -u
O=gpurun_out
T=${1:-r5w}
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for v in d 1 2 3 4; do
    for n in 650 50; do
      if [ $v = d ]; then unset TTS_CODEC_X3P_TILE; else export TTS_CODEC_X3P_TILE=$v; fi
      timeout -k 10 120 python scripts/codec_probe32.py 1 $n 2>&1 | grep codes >> $O/${T}_ab_codec1_tile.txt || exit $?
      echo "  (TTS_CODEC_X3P_TILE=$v)" >> $O/${T}_ab_codec1_tile.txt
    done
  done
done
cat $O/${T}_ab_codec1_tile.txt
