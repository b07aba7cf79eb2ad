#!/bin/bash
# r6a: (1) lead combine form 2 (scripts/experiments/lead_combine, built as ablib/lib_lead.so)
# A/B at 32 and 24 rows, ids md5 must match; (2) the RCCL path at one rank with the new
# TTS-1-Max sharded line; (3) prefill kernel stats at 1 and 32 prompts; (4) the GPU suite
# (new: switch bit-identity, K = 768 norm fallback, 4 GiB refusal).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
TTS_LIB_PATH=ablib/lib_lead.so timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_LEAD_COMBINE 32 3 > $OUT/r6a_lead_32.txt 2>&1; rc=$?; tail -6 $OUT/r6a_lead_32.txt; fatal $rc lead32
TTS_LIB_PATH=ablib/lib_lead.so timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_LEAD_COMBINE 24 2 > $OUT/r6a_lead_24.txt 2>&1; rc=$?; tail -4 $OUT/r6a_lead_24.txt; fatal $rc lead24
TTS_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/r6a_dist1.json 2> $OUT/r6a_dist1.err; rc=$?; tail -3 $OUT/r6a_dist1.err; fatal $rc dist1
for n in 1 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r6a_prefill$n -o run -- python3 scripts/prefill_probe.py $n > $OUT/r6a_prefill$n.log 2>&1; rc=$?; tail -2 $OUT/r6a_prefill$n.log; fatal $rc prefill$n
  find $OUT/r6a_prefill$n -name "*trace*" -delete
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > $OUT/r6a_tests.log 2>&1; rc=$?; tail -5 $OUT/r6a_tests.log; fatal $rc tests
