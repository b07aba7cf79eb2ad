#!/bin/bash
# round 5, session e: GPU suite on the buffer-load weight stream + the planes codec GEMM
# (gemm_x3p); codec A/B (TTS_CODEC_X3P 0/1: time + waveform md5); LM A/B against the r5a
# library (1 / 32 rows TTS-1, 8 rows TTS-1-Max); the bs=32 decode step's kernel stats;
# TTS-1-Max 8-row stamps and the RMSNorm-prologue bound (diagnostic build)
set -u
O=gpurun_out
T=${1:-r5e}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for v in 0 1; do
  for b in 32 1; do
    TTS_CODEC_X3P=$v timeout -k 10 120 python scripts/codec_probe32.py $b 650 >> $O/${T}_ab_codec.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P=$v)" >> $O/${T}_ab_codec.txt
  done
done
cat $O/${T}_ab_codec.txt
export AB_V0=$PWD/ablib/lib_r5a.so AB_V1=$PWD/ablib/lib_cur.so
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 1 1 > $O/${T}_ab_1.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 32 1 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_1.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
unset AB_V0 AB_V1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof32 -o run -- \
  python3 scripts/gen_probe.py 32 500 > $O/${T}_prof32.log 2>&1 || exit $?
find $O/${T}_prof32 -name "*trace*" -delete
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 || exit $?
export AB_V0=0 AB_V1=16 TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_WGEMM_DIAG 8 1 > $O/${T}_ab_nonorm_max8.txt 2>&1
rc=$?
cat $O/${T}_ab_nonorm_max8.txt
exit $rc
