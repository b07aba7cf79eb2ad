#!/bin/bash
# round 6: the screen with four 8 KiB stages in flight per wave (-DTTS_SCR_R=4) vs two
set -u
O=gpurun_out
T=${1:-r6ah}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
L=tts-max_amd/tts_amd
for r in 1 8 32; do
  AB_V0=$L/libtts_mi355x.so AB_V1=$L/libtts_r4.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH $r 2 > $O/${T}_ab_r4_$r.txt 2>&1; rc=$?
  cat $O/${T}_ab_r4_$r.txt; fatal $rc r4_$r
done
AB_ARCH=tts1-max AB_V0=$L/libtts_mi355x.so AB_V1=$L/libtts_r4.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_r4_max8.txt 2>&1; rc=$?
cat $O/${T}_ab_r4_max8.txt; fatal $rc r4_max8
echo done
