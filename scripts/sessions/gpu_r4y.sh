#!/bin/bash
# round-4 final measurement: GPU suite, smoke, the bench line + rocprof stats, the TTS-1-Max
# shard (configs[3]) with rocprof stats, PMC of the 8-row fused QKV + attention + o_proj launch
set -u
O=gpurun_out
T=${1:-r4y}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_bench_tts1max_bs8.json 2> $O/${T}_bench_tts1max.err && \
find $O/${T}_prof_max -name "*trace*" -delete && \
ARCH=tts1-max bash scripts/pmc_traffic.sh qkv_attn_oproj 8 > /dev/null 2>&1 && \
bash scripts/pmc_traffic.sh qkv_attn_oproj 8 > /dev/null 2>&1
rc=$?
echo "rc=$rc"
exit $rc
