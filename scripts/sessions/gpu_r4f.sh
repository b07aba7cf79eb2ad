#!/bin/bash
# round-4 measurement: rocprof kernel stats of the bench (bs=1 + secondaries) and of the
# TTS-1-Max shard, PMC HBM traffic of the decode kernels at 1 / 32 rows (TTS-1) and 8 rows
# (TTS-1-Max), MFMA utilisation of the codec and prefill GEMMs
set -u
O=gpurun_out
T=${1:-r4f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/${T}_prof_bench.json 2> $O/${T}_prof_bench.err && \
find $O/${T}_prof -name "*trace*" -delete && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_prof_max_bench.json 2> $O/${T}_prof_max_bench.err && \
find $O/${T}_prof_max -name "*trace*" -delete && \
for kr in "qkv 32" "o_proj 32" "gate_up 32" "down 32" "attention 32" "gate_up 1" "down 1" "qkv_attn_oproj 1" "lm_head 1"; do
  bash scripts/pmc_traffic.sh $kr > /dev/null 2>&1 || { echo "pmc $kr failed"; exit 1; }
done && \
for kr in "qkv_attn 8" "o_proj 8" "gate_up 8" "down 8" "lm_head 8"; do
  ARCH=tts1-max bash scripts/pmc_traffic.sh $kr > /dev/null 2>&1 || { echo "pmc max $kr failed"; exit 1; }
done && \
bash scripts/mfma_util.sh > $O/${T}_mfma.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
