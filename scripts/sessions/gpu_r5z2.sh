#!/bin/bash
# round-5 final measurement, second pass (after the lone-utterance tile heuristic): GPU suite,
# smoke, bench line + rocprof stats; lone-utterance codec A/B against session i's library
set -u
O=gpurun_out
T=${1:-r5z2}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
for r in 0 1; do
  for lib in $PWD/ablib/lib_r5i.so $PWD/tts-max_amd/tts_amd/libtts_mi355x.so; do
    for n in 650 50; do
      TTS_LIB_PATH=$lib timeout -k 10 120 python scripts/codec_probe32.py 1 $n 2>&1 | grep codes >> $O/${T}_ab_codec1_heur.txt || exit $?
      echo "  ($(basename $lib))" >> $O/${T}_ab_codec1_heur.txt
    done
  done
done
cat $O/${T}_ab_codec1_heur.txt
