#!/bin/bash
# round 5, session d: codec GPU tests + codec A/B on the embed-conv planes; the bs=32 decode
# step's kernel stats (rocprofv3); TTS-1-Max 8-row stamps and the RMSNorm-prologue bound
set -u
O=gpurun_out
T=${1:-r5d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_config1.py tests/test_gpu_streaming.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/${T}_codec_tests.log 2>&1; rc=$?; tail -3 $O/${T}_codec_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    for b in 32 1; do
      TTS_CODEC_X3P=$v timeout -k 10 120 python scripts/codec_probe32.py $b 650 >> $O/${T}_ab_codec.txt 2>&1 || exit $?
      echo "  (TTS_CODEC_X3P=$v)" >> $O/${T}_ab_codec.txt
    done
  done
done
cat $O/${T}_ab_codec.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof32 -o run -- \
  python3 scripts/gen_probe.py 32 500 > $O/${T}_prof32.log 2>&1 || exit $?
find $O/${T}_prof32 -name "*trace*" -delete
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 || exit $?
export AB_V0=0 AB_V1=16 TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so
AB_ARCH=tts1-max timeout -k 10 600 python scripts/env_ab_probe.py TTS_WGEMM_DIAG 8 1 > $O/${T}_ab_nonorm_max8.txt 2>&1
rc=$?
cat $O/${T}_ab_nonorm_max8.txt
exit $rc
