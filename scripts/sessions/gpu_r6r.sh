#!/bin/bash
# round-6 final measurement of the final library: GPU suite, smoke, the bench line + rocprof
# kernel stats, and the RCCL path at one rank (rank 0's stdout must be the one JSON line)
set -u
O=gpurun_out
T=${1:-r6r}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
TTS_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29563 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_dist1.json 2> $O/${T}_dist1.err || exit $?
wc -l $O/${T}_dist1.json
echo done
