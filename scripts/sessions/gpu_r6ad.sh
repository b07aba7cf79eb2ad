#!/bin/bash
# round 6: what the screen's stream costs at 32 / 1 rows: probe builds without the MFMAs (1),
# without the per-unit epilogue (2), without both (3) vs the library (timing only: wrong ids)
set -u
O=gpurun_out
T=${1:-r6ad}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
L=tts-max_amd/tts_amd
export TTS_HEAD_SCREEN_DIAG=1  # (both sides skip the recompute: the stream alone)
for v in 1 2 3; do
  AB_V0=$L/libtts_mi355x.so AB_V1=$L/libtts_probe$v.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH 32 1 > $O/${T}_probe${v}_32.txt 2>&1; rc=$?
  cat $O/${T}_probe${v}_32.txt; fatal $rc probe$v
done
AB_V0=$L/libtts_mi355x.so AB_V1=$L/libtts_probe3.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH 1 1 > $O/${T}_probe3_1.txt 2>&1; rc=$?
cat $O/${T}_probe3_1.txt; fatal $rc probe3_1
echo done
