#!/bin/bash
# round 5, session f: GPU suite (single-unit stream path, contraction-free plane split);
# codec A/B + rocprof stats of both codec paths; LM A/B vs r5a; the RCCL path rehearsed at one
# rank (TTS_BENCH_DIST=1 under torch.distributed.run) beside the plain line
set -u
O=gpurun_out
T=${1:-r5f}
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for v in 0 1; do
  for b in 32 1; do
    TTS_CODEC_X3P=$v timeout -k 10 120 python scripts/codec_probe32.py $b 650 >> $O/${T}_ab_codec.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P=$v)" >> $O/${T}_ab_codec.txt
  done
done
cat $O/${T}_ab_codec.txt
for v in 0 1; do
  TTS_CODEC_X3P=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_codec$v -o run -- \
    python3 scripts/codec_probe32.py 32 650 > $O/${T}_prof_codec$v.log 2>&1 || exit $?
  find $O/${T}_prof_codec$v -name "*trace*" -delete
done
export AB_V0=$PWD/ablib/lib_r5a.so AB_V1=$PWD/ablib/lib_cur.so
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 1 2 > $O/${T}_ab_1.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 32 2 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_1.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
unset AB_V0 AB_V1
timeout -k 10 300 python bench.py --steps 3 --no-secondary --no-cpu-baseline > $O/${T}_bench_plain.json 2> $O/${T}_bench_plain.err || exit $?
TTS_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --steps 3 --no-secondary --no-cpu-baseline > $O/${T}_bench_rccl_rank1.json 2> $O/${T}_bench_rccl.err
rc=$?
cat $O/${T}_bench_plain.json $O/${T}_bench_rccl_rank1.json | cut -c1-400
exit $rc
