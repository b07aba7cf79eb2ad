#!/bin/bash
# round 6: the prefill GEMM in canonical K chunks (one chunk per workgroup for short prompts,
# the running sum in registers otherwise) and the XCD-grouped tile order: the GPU suite, the
# prefill A/B against the frozen round-6 base library (ablib/lib_r6base.so), and the prefill
# kernel stats at 1 and 32 prompts
set -u
O=gpurun_out
T=${1:-r6i}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -4 $O/${T}_tests.log; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/prefill_ab.py 2 TTS_LIB_PATH=ablib/lib_r6base.so - TTS_PGEMM_XCD=0 TTS_PGEMM_SPLIT=0 TTS_PGEMM_SPLIT=2 > $O/${T}_prefill_ab.txt 2>&1; rc=$?
cat $O/${T}_prefill_ab.txt; fatal $rc prefill_ab
for n in 1 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prefill$n -o run -- python3 scripts/prefill_probe.py $n > $O/${T}_prefill$n.log 2>&1; rc=$?; tail -2 $O/${T}_prefill$n.log; fatal $rc prefill$n
  find $O/${T}_prefill$n -name "*trace*" -delete
done
echo done
