#!/bin/bash
# round-4: batched-decode parity on the new paths, same-box A/Bs, stamps, codec GEMM rates,
# TTS-1-Max kernel profile
set -u
O=gpurun_out
T=${1:-r4c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lm.py tests/test_gpu_chain.py tests/test_gpu_chain_max.py tests/test_gpu_tts1max.py -m gpu > $O/${T}_tests.log 2>&1 && \
cp $O/long_tf_dev_lm_tts1_long.json $O/${T}_long_tf_dev_lm_tts1_long.json && cp $O/long_tf_dev_lm_max2l_long.json $O/${T}_long_tf_dev_lm_max2l_long.json && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_AGR32 32 2 > $O/${T}_ab_agr32.txt 2>&1 && \
AB_V0=1 AB_V1=6 timeout -k 10 600 python scripts/env_ab_probe.py TTS_ATTN_SPLIT 32 2 > $O/${T}_ab_split32.txt 2>&1 && \
AB_V0=1 AB_V1=6 timeout -k 10 600 python scripts/env_ab_probe.py TTS_ATTN_SPLIT 8 2 > $O/${T}_ab_split8.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_NORM32 32 2 > $O/${T}_ab_norm32.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_CSPLIT32 32 2 > $O/${T}_ab_csplit32.txt 2>&1 && \
timeout -k 10 600 python scripts/env_ab_probe.py TTS_COMBINE_FIXED 32 2 > $O/${T}_ab_combine32.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 450 32 > $O/${T}_stamps32.txt 2>&1 && \
timeout -k 10 300 python scripts/codec_gemm_probe.py > $O/${T}_codec_gemm.txt 2>&1 && \
for tl in 0 1 2 0 1 2; do TTS_CODEC_TILE=$tl timeout -k 10 120 python scripts/codec_probe32.py 32 650 | sed "s/^/tile $tl: /" >> $O/${T}_ab_codec_tile.txt || exit 1; done && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec.py -m gpu > $O/${T}_codec_tests.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $O/${T}_bench_max.json 2> $O/${T}_bench_max.err
rc=$?
find $O/${T}_prof_max -name "*trace*" -delete 2>/dev/null
echo "rc=$rc"
exit $rc
