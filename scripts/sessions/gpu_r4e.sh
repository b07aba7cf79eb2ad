#!/bin/bash
# round-4: batched fused QKV+attention, K-sliced 32-row projections, codec A planes: parity, A/Bs, bench
set -u
O=gpurun_out
T=${1:-r4e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_launch.py tests/test_gpu_lm.py tests/test_gpu_chain.py tests/test_gpu_chain_max.py tests/test_gpu_tts1max.py tests/test_gpu_ops.py tests/test_gpu_codec.py -m gpu > $O/${T}_tests.log 2>&1 && \
cp $O/long_tf_dev_lm_tts1_long.json $O/${T}_long_tf_dev_lm_tts1_long.json && cp $O/long_tf_dev_lm_max2l_long.json $O/${T}_long_tf_dev_lm_max2l_long.json && \
AB_V0=0 AB_V1=16 timeout -k 10 600 python scripts/env_ab_probe.py TTS_FATTN_ROWS 8 2 > $O/${T}_ab_fattn_rows8.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_KSLICE32 32 2 > $O/${T}_ab_kslice32.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_QKV_DEFER 32 2 > $O/${T}_ab_qkvdefer32.txt 2>&1 && \
for v in 1 0 1 0; do TTS_CODEC_EXPF=$v timeout -k 10 120 python scripts/codec_probe32.py 32 650 | sed "s/^/expf $v: /" >> $O/${T}_ab_codec_expf.txt || exit 1; done && \
for v in 0 1 0 1; do TTS_CODEC_APRE=$v timeout -k 10 120 python scripts/codec_probe32.py 32 650 | sed "s/^/apre $v: /" >> $O/${T}_ab_codec_apre.txt || exit 1; done && \
TTS_CODEC_APRE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -m gpu > $O/${T}_codec_apre_tests.log 2>&1 && \
TTS_FATTN_ROWS=0 timeout -k 10 600 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_bench_max_sep.json 2> $O/${T}_bench_max_sep.err && \
timeout -k 10 600 python bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline --no-secondary > $O/${T}_bench_max.json 2> $O/${T}_bench_max.err && \
timeout -k 10 900 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err
rc=$?
echo "rc=$rc"
exit $rc
