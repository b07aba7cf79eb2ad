#!/bin/bash
# round-6 final measurement, part 1 (the committed library, in-tree): GPU suite, smoke, the
# bench line (default workload + secondaries + CPU baseline) and its rocprofv3 kernel stats
set -u
T=${1:-r6g}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests smoke bench prof || exit $?
echo done
