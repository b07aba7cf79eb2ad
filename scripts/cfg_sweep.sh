#!/bin/bash
# wgemm launch-shape sweep at the TTS-1 decode shapes (one process per forced shape)
for cfg in -1 0 1 3 4 5 6; do
  echo "== TTS_WGEMM_CFG=$cfg"
  TTS_WGEMM_CFG=$cfg timeout -k 10 120 python scripts/microbench.py --wgemm-only 2>/dev/null || exit $?
done
