#!/bin/bash
# round 5, session l: codec attention with conflict-free 160-B K / V^T rows (bits unchanged);
# 128-query workgroups A/B; 32 rows: o_proj unsliced + the gate/up RMSNorm in its (now batched)
# LDS prologue vs the K-sliced o_proj + combine launch
set -u
O=gpurun_out
T=${1:-r5l}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_streaming.py -m gpu > $O/${T}_codec_tests.log 2>&1 || exit $?
tail -2 $O/${T}_codec_tests.log
for r in 0 1; do
  for lib in $PWD/ablib/lib_r5i.so $PWD/tts-max_amd/tts_amd/libtts_mi355x.so; do
    TTS_LIB_PATH=$lib timeout -k 10 120 python scripts/codec_probe32.py 32 650 2>&1 | grep codes >> $O/${T}_ab_codec_attn.txt || exit $?
    echo "  ($(basename $lib))" >> $O/${T}_ab_codec_attn.txt
  done
  TTS_CODEC_ATTN_W=8 timeout -k 10 120 python scripts/codec_probe32.py 32 650 2>&1 | grep codes >> $O/${T}_ab_codec_attn.txt || exit $?
  echo "  (TTS_CODEC_ATTN_W=8)" >> $O/${T}_ab_codec_attn.txt
done
cat $O/${T}_ab_codec_attn.txt
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/${T}_apmc -o pmc -- \
  python3 scripts/codec_probe32.py 32 650 > $O/${T}_apmc.log 2>&1 || exit $?
python3 scripts/pmc_kernels.py "codec_attn_kernel<[^>]*>|gemm_x3p_kernel<[^>]*>" /tmp/${T}_apmc > $O/${T}_pmc_codec_attn.json
grep -E "kernel|mfma_util|conflict" $O/${T}_pmc_codec_attn.json
export AB_V0=1 AB_V1=0
TTS_NORM32=1 timeout -k 10 400 python scripts/env_ab_probe.py TTS_KSLICE32_RESID 32 2 > $O/${T}_ab_oproj32_norm32.txt 2>&1
rc=$?
cat $O/${T}_ab_oproj32_norm32.txt
exit $rc
