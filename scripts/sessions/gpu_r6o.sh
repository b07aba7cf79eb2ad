#!/bin/bash
# round 6: deeper DMA rings for the lone utterance's 128 x 64 codec tiles (c_attn, fc1) and the
# four-stage one-wave tiles: codec A/B (one 650-code utterance, 32 x 650)
set -u
O=gpurun_out
T=${1:-r6o}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u scripts/codec_ab.py 2 - TTS_CODEC_NS_128X64=3 TTS_CODEC_NS_128X64=4 TTS_CODEC_X3P_SMALL4=1 TTS_CODEC_NS_128X64=4,TTS_CODEC_X3P_SMALL4=1 > $O/${T}_codec_ab.txt 2>&1; rc=$?
cat $O/${T}_codec_ab.txt; fatal $rc codec_ab
echo done
