#!/bin/bash
# round-6 final measurement with the screened lm_head: GPU suite, smoke, the bench line + rocprof
# kernel stats; the TTS-1-Max configs[3] shard line + stats; PMC HBM traffic of the screened head
# (TTS-1 1 / 32 rows, TTS-1-Max 8 rows); the RCCL path at one rank
set -u
O=gpurun_out
T=${1:-r6ag}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_bench_tts1max_bs8.json 2> $O/${T}_bench_tts1max.err || exit $?
find $O/${T}_prof_max -name "*trace*" -delete
cat $O/${T}_bench_tts1max_bs8.json | head -c 600; echo
for kr in "head_screened 1" "head_screened 32"; do
  bash scripts/pmc_traffic.sh $kr > /dev/null 2>&1 || exit $?
done
ARCH=tts1-max bash scripts/pmc_traffic.sh head_screened 8 > /dev/null 2>&1 || exit $?
ls $O/pmc/*.json
TTS_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29563 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_dist1.json 2> $O/${T}_dist1.err || exit $?
head -c 400 $O/${T}_dist1.json; echo
echo done
