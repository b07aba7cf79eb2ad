#!/bin/bash
# round 6: prefill rope + KV append (q/k per row, V^T per query block through LDS): the
# GPU suite, the prefill A/B vs the committed library (ablib/lib_r6m.so), prefill kernel stats
set -u
O=gpurun_out
T=${1:-r6q}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -4 $O/${T}_tests.log; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/prefill_ab.py 2 TTS_LIB_PATH=ablib/lib_r6m.so - > $O/${T}_prefill_ab.txt 2>&1; rc=$?
cat $O/${T}_prefill_ab.txt; fatal $rc prefill_ab
for n in 1 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prefill$n -o run -- python3 scripts/prefill_probe.py $n > $O/${T}_prefill$n.log 2>&1; rc=$?; tail -2 $O/${T}_prefill$n.log; fatal $rc prefill$n
  find $O/${T}_prefill$n -name "*trace*" -delete
done
echo done
