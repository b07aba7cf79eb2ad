#!/bin/bash
# round 5, session b: GPU suite on the buffer-load weight stream, then same-box A/B against the
# r5a library at 1 / 32 rows (TTS-1) and 8 rows (TTS-1-Max)
set -u
O=gpurun_out
T=${1:-r5b}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
export AB_V0=$PWD/ablib/lib_r5a.so AB_V1=$PWD/ablib/lib_buf.so
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 1 2 > $O/${T}_ab_1.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 32 2 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 600 python scripts/env_ab_probe.py TTS_LIB_PATH 8 2 > $O/${T}_ab_max8.txt 2>&1
rc=$?
cat $O/${T}_ab_*.txt
exit $rc
