#!/bin/bash
# round 5, session v: where a lone 650-code utterance's codec pass goes (kernel trace: per-kernel
# totals and the idle time between launches)
set -u
O=gpurun_out
T=${1:-r5v}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_c1 -o run -- \
  python3 scripts/codec_probe32.py 1 650 > $O/${T}_c1.log 2>&1 || exit $?
python3 scripts/trace_gaps.py $(find /tmp/${T}_c1 -name "*kernel_trace.csv" | head -1) --burst-gap 300 > $O/${T}_codec1_gaps.txt
cp $(find /tmp/${T}_c1 -name "*kernel_stats.csv" | head -1) $O/${T}_codec1_kernel_stats.csv
python3 scripts/kstats.py $O/${T}_codec1_kernel_stats.csv 16
tail -30 $O/${T}_codec1_gaps.txt
