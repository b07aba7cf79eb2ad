#!/bin/bash
# round 6: the screened head's parity tests incl. heavy-tailed lm_head weights
set -u
O=gpurun_out
T=${1:-r6al}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_head_screen.py -v -rf --timeout 400 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -8 $O/${T}_tests.log; exit $rc
