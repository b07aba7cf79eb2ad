#!/bin/bash
# GPU-box check of the tree: the -m gpu suite, then one default bench line (with the CPU
# baseline) and a rocprofv3 kernel-stats pass of a short bench.  Each GPU step has its own
# time limit and the script stops at the first failure.   usage: scripts/gpu_check.sh TAG [steps...]
set -u
TAG=$1; shift
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf \
             > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
           tail -2 $OUT/${TAG}_tests.log ;;
    bench) timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
             || { tail -20 $OUT/${TAG}_bench.err; exit 1; }
           cat $OUT/${TAG}_bench.json ;;
    quick) timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${TAG}_quick.json 2> $OUT/${TAG}_quick.err \
             || { tail -20 $OUT/${TAG}_quick.err; exit 1; }
           cat $OUT/${TAG}_quick.json ;;
    prof)  D=/tmp/prof_$TAG
           timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
             python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1 || { tail -20 $OUT/${TAG}_prof.log; exit 1; }
           cp $D/run_kernel_stats.csv $OUT/${TAG}_kernel_stats.csv; head -25 $OUT/${TAG}_kernel_stats.csv | cut -c1-160 ;;
  esac
done
