#!/bin/bash
# A/B of decode-step cache warming in one GPU session (same device): bench with and without.
set -u
OUT=gpurun_out; TAG=${1:-ab}
mkdir -p $OUT
for pf in 1 0 1 0; do
  TTS_PREFETCH=$pf timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_pf${pf}.json 2>/dev/null; rc=$?
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc"; exit $rc; fi
  python3 -c "import json;d=json.load(open('$OUT/${TAG}_pf${pf}.json'));print('pf=$pf', d['value'], d['roofline']['decode_step'])"
done
