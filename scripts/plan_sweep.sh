#!/bin/bash
# Stream-plan sweep (scripts/wgemm_probe): launch shapes of lm_gemm.hip's table forced on
# every decode matrix they fit (TTS_STREAM_PLAN=<shape>[,grid]), and diagnostic switches
# (TTS_WGEMM_DIAG).  Run on the GPU box.   usage: scripts/plan_sweep.sh "<plans>" "<diags>"
PLANS=${1:-"default 0 1 2 3 4 5 6 0,512 0,1024"}
DIAGS=${2:-"0"}
for d in $DIAGS; do
  for c in $PLANS; do
    echo "== plan $c diag $d"
    if [ "$c" = default ]; then TTS_WGEMM_DIAG=$d timeout -k 10 100 ./scripts/wgemm_probe || exit $?
    else TTS_STREAM_PLAN=$c TTS_WGEMM_DIAG=$d timeout -k 10 100 ./scripts/wgemm_probe || exit $?; fi
  done
done
