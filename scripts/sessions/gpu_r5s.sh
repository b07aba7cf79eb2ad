#!/bin/bash
# round 5, session s: the lone utterance's one-wave codec GEMM tiles with four stages (the DMA
# three steps ahead, TTS_CODEC_X3P_SMALL4=1) against the two-stage form; the codec GEMM forms'
# bit-equality test
set -u
O=gpurun_out
T=${1:-r5s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_codec.py -m gpu -k schedules > $O/${T}_sched_tests.log 2>&1 || exit $?
tail -10 $O/${T}_sched_tests.log
for r in 0 1; do
  for v in 0 1; do
    for b in 1 8; do
      TTS_CODEC_X3P_SMALL4=$v timeout -k 10 120 python scripts/codec_probe32.py $b 650 2>&1 | grep codes >> $O/${T}_ab_codec_small4.txt || exit $?
      echo "  (TTS_CODEC_X3P_SMALL4=$v)" >> $O/${T}_ab_codec_small4.txt
    done
  done
done
cat $O/${T}_ab_codec_small4.txt
