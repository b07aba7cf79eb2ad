#!/bin/bash
# rocprofv3 kernel-trace --stats of one bench run; the (large) trace stays in /tmp on the box,
# only the per-kernel stats summary is kept under gpurun_out/.   usage: scripts/prof_stats.sh TAG [bench args]
set -u
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-secondary "$@" > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_prof.log
cp $D/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv 2>/dev/null
exit $rc
