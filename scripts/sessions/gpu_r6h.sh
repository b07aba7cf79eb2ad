#!/bin/bash
# round-6 final measurement, part 2: the TTS-1-Max shard (configs[3]) line + rocprof stats, the
# RCCL path at one rank with the configs[3] line, and PMC HBM traffic of the bench's kernels
# (bs 1, 32) and of the TTS-1-Max 8-row launches (scripts/pmc_traffic.sh)
set -u
O=gpurun_out
T=${1:-r6h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_bench_tts1max_bs8.json 2> $O/${T}_bench_tts1max.err || exit $?
find $O/${T}_prof_max -name "*trace*" -delete
for kr in "gate_up 1" "down 1" "qkv_attn_oproj 1" "lm_head 1" "gate_up 32" "qkv 32" "o_proj 32" "down 32" "attention 32"; do
  bash scripts/pmc_traffic.sh $kr > /dev/null 2>&1 || exit $?
done
for kr in "qkv_attn_oproj 8" "gate_up 8" "down 8"; do
  ARCH=tts1-max bash scripts/pmc_traffic.sh $kr > /dev/null 2>&1 || exit $?
done
ls $O/pmc/*.json
TTS_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29563 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_dist1.json 2> $O/${T}_dist1.err || exit $?
echo done
