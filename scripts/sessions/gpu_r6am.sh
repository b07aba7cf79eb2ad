#!/bin/bash
# round 6: one-row screen without the read of the other shards' bounds (no wait at one row) vs with
set -u
O=gpurun_out
T=${1:-r6am}
mkdir -p $O
export TMPDIR=/tmp
L=tts-max_amd/tts_amd
AB_V0=$L/libtts_base.so AB_V1=$L/libtts_mi355x.so timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_LIB_PATH 1 3 > $O/${T}_ab_shardread_1.txt 2>&1; rc=$?
cat $O/${T}_ab_shardread_1.txt; exit $rc
