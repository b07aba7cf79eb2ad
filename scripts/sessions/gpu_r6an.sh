#!/bin/bash
# round-6 closing measurement: the whole GPU suite, smoke and the bench line + rocprof kernel stats
# screened lm_head
set -u
O=gpurun_out
T=${1:-r6an}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
echo done
