#!/bin/bash
# round 6: the LDS-DMA ring prefill GEMM for long batched prefill (M > 512): the GPU suite, the
# prefill A/B (round-6 base library; the register-staged tall kernel; forced gate/up tiles at one
# prompt), prefill kernel stats at 32 prompts
set -u
O=gpurun_out
T=${1:-r6l}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -4 $O/${T}_tests.log; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 900 python -u scripts/prefill_ab.py 2 TTS_LIB_PATH=ablib/lib_r6base.so - TTS_PGEMM_RING=0 TTS_PGEMM_TILE=44 TTS_PGEMM_TILE=42 TTS_PGEMM_TILE=22 > $O/${T}_prefill_ab.txt 2>&1; rc=$?
cat $O/${T}_prefill_ab.txt; fatal $rc prefill_ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prefill32 -o run -- python3 scripts/prefill_probe.py 32 > $O/${T}_prefill32.log 2>&1; rc=$?; tail -2 $O/${T}_prefill32.log; fatal $rc prefill32
find $O/${T}_prefill32 -name "*trace*" -delete
echo done
