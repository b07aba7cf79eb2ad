#!/bin/bash
# round 6: the screened lm_head at 17..32 rows (rows quantised once by head_rowquant_kernel, the
# int8 image alone in LDS, two m-tiles in the exact recompute): parity tests + same-bits
# switches, A/B vs the full lm_head at 24 / 32 rows, the bench line
set -u
O=gpurun_out
T=${1:-r6aa}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_head_screen.py tests/test_gpu_switches.py -k "head or HEAD" -v -rf --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -12 $O/${T}_tests.log; fatal $rc tests
for r in 32 8 1; do
  timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN $r 2 > $O/${T}_ab_head_screen_$r.txt 2>&1; rc=$?
  cat $O/${T}_ab_head_screen_$r.txt; fatal $rc ab$r
done
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err; rc=$?
tail -3 $O/${T}_bench.err; cat $O/${T}_bench.json; fatal $rc bench
echo done
