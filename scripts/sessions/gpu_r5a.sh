#!/bin/bash
# round 5, session a: GPU suite + bench after the stream-issue / ring-drain fixes, then the
# TTS-1-Max shard (configs[3]) bench line
set -u
O=gpurun_out
T=${1:-r5a}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests bench || exit $?
timeout -k 10 600 python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary \
  > $O/${T}_bench_tts1max_bs8.json 2> $O/${T}_bench_tts1max.err
rc=$?
cat $O/${T}_bench_tts1max_bs8.json
echo "rc=$rc"
exit $rc
