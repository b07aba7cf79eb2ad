#!/bin/bash
# round-4: stamps of the fused 2..16-row QKV + attention + o_proj launch
set -u
O=gpurun_out
T=${1:-r4t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/stamp_probe.py 452 8 tts1-max > $O/${T}_stamps_max8.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 8 > $O/${T}_stamps_tts1_8.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 452 2 > $O/${T}_stamps_tts1_2.txt 2>&1
rc=$?
echo "rc=$rc"
exit $rc
