#!/bin/bash
# round 5, session j: GPU suite with the codec GEMM's LDS-transposed epilogue; codec A/B against
# session i's library (same box), the stamps-build phase split again
set -u
O=gpurun_out
T=${1:-r5j}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for r in 0 1; do
  for lib in $PWD/ablib/lib_r5i.so $PWD/tts-max_amd/tts_amd/libtts_mi355x.so; do
    for b in 32 1; do
      TTS_LIB_PATH=$lib timeout -k 10 120 python scripts/codec_probe32.py $b 650 2>&1 | grep codes >> $O/${T}_ab_codec_epi.txt || exit $?
      echo "  ($(basename $lib))" >> $O/${T}_ab_codec_epi.txt
    done
  done
done
cat $O/${T}_ab_codec_epi.txt
TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so TTS_CODEC_STAMPS=1 timeout -k 10 120 \
  python scripts/codec_probe32.py 32 650 2>&1 | grep -v amdgpu.ids > $O/${T}_codec_stamps.txt || exit $?
cat $O/${T}_codec_stamps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_codec -o run -- \
  python3 scripts/codec_probe32.py 32 650 > $O/${T}_prof_codec.log 2>&1 || exit $?
find $O/${T}_prof_codec -name "*trace*" -delete
python3 scripts/kstats.py $(find $O/${T}_prof_codec -name "*kernel_stats.csv" | head -1) 12
