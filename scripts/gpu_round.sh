#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.  Every GPU step has its
# own time limit; a crash/timeout (exit >= 124) ends the script before any further GPU work.
# usage: scripts/gpu_round.sh TAG [tests|smoke|bench|bench32|prof]...
set -u
TAG=${1:-r1}; shift
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $2; stopping"; exit $rc; fi; }
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1; rc=$?
      tail -5 $OUT/${TAG}_tests.log; stop_if_fatal $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1; rc=$?
      tail -3 $OUT/${TAG}_smoke.log; stop_if_fatal $rc smoke ;;
    bench)
      timeout -k 10 900 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err; rc=$?
      tail -3 $OUT/${TAG}_bench.err; cat $OUT/${TAG}_bench.json; stop_if_fatal $rc bench ;;
    bench32)
      timeout -k 10 900 python bench.py --batch 32 --no-cpu-baseline > $OUT/${TAG}_bench32.json 2> $OUT/${TAG}_bench32.err; rc=$?
      tail -3 $OUT/${TAG}_bench32.err; cat $OUT/${TAG}_bench32.json; stop_if_fatal $rc bench32 ;;
    prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run -- \
        python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_prof.log 2>&1; rc=$?
      tail -3 $OUT/${TAG}_prof.log; find $OUT/${TAG}_prof -name "*trace*" -delete; find $OUT/${TAG}_prof -name "*stats*"; stop_if_fatal $rc prof ;;
  esac
done
