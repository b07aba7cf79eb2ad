#!/bin/bash
# round-5 re-measure after the 17..32-row four-stage gate/up ring: suite, smoke, bench + rocprof,
# PMC of the 32-row gate/up
set -u
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh r5z4 tests smoke bench prof || exit $?
bash scripts/pmc_traffic.sh gate_up 32 > /dev/null 2>&1 || exit $?
ls $O/pmc/*.json
echo done
