#!/bin/bash
# round-4: bs=32 K-sliced qkv/o_proj (TTS_KSLICE32) parity + same-box A/B + bench
set -u
O=gpurun_out
T=${1:-r4d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lm.py tests/test_gpu_chain.py tests/test_gpu_ops.py -m gpu > $O/${T}_tests.log 2>&1 && \
cp $O/long_tf_dev_lm_tts1_long.json $O/${T}_long_tf_dev_lm_tts1_long.json && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_KSLICE32 32 2 > $O/${T}_ab_kslice32.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_KSLICE32 24 1 > $O/${T}_ab_kslice24.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_QKV_DEFER 32 2 > $O/${T}_ab_qkvdefer32.txt 2>&1 && \
for v in 0 1 0 1; do TTS_CODEC_APRE=$v timeout -k 10 120 python scripts/codec_probe32.py 32 650 | sed "s/^/apre $v: /" >> $O/${T}_ab_codec_apre.txt || exit 1; done && \
TTS_CODEC_APRE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -m gpu > $O/${T}_codec_apre_tests.log 2>&1 && \
timeout -k 10 900 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err
rc=$?
echo "rc=$rc"
exit $rc
