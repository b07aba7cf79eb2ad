#!/bin/bash
# round-4 diagnostics: batched-decode stamps, TTS-1-Max kernel profile, codec GEMM rates
set -u
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lm.py tests/test_gpu_chain.py tests/test_gpu_chain_max.py tests/test_gpu_tts1max.py -m gpu > $O/r4b_tests.log 2>&1 && \
cp $O/long_tf_dev_lm_tts1_long.json $O/r4b_long_tf_dev_lm_tts1_long.json && cp $O/long_tf_dev_lm_max2l_long.json $O/r4b_long_tf_dev_lm_max2l_long.json && \
timeout -k 10 300 python scripts/stamp_probe.py 450 32 > $O/r4b_stamps32.txt 2>&1 && \
timeout -k 10 300 python scripts/stamp_probe.py 450 1 > $O/r4b_stamps1.txt 2>&1 && \
timeout -k 10 300 python scripts/codec_gemm_probe.py > $O/r4b_codec_gemm.txt 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r4b_prof_max -o run -- \
  python3 bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $O/r4b_bench_max.json 2> $O/r4b_bench_max.err
rc=$?
find $O/r4b_prof_max -name "*trace*" -delete 2>/dev/null
echo "rc=$rc"
exit $rc
