#!/bin/bash
# round 6: codec running sum only where K spans more than one canonical chunk (template CH):
# codec tests, codec A/B vs the round-6 base library, codec kernel stats of one utterance
set -u
O=gpurun_out
T=${1:-r6k}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_config1.py -m gpu -v -rf --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1; rc=$?
tail -4 $O/${T}_tests.log; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/codec_ab.py 2 TTS_LIB_PATH=ablib/lib_r6base.so - TTS_CODEC_SPLIT=0 > $O/${T}_codec_ab.txt 2>&1; rc=$?
cat $O/${T}_codec_ab.txt; fatal $rc codec_ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_codec1 -o run -- python3 scripts/codec_probe.py 650 1 > $O/${T}_codec1.log 2>&1; rc=$?; tail -2 $O/${T}_codec1.log; fatal $rc codec1
find $O/${T}_codec1 -name "*trace*" -delete
echo done
