#!/bin/bash
# round 5, session i: GPU suite on the reverted RMSNorm / attention prologues (r5f's, with the
# 32-bit fragment offsets at head dim 64) and the codec GEMM with early interleaved DMA on the
# big tiles; codec A/B (ILV forced off / default), LM A/B against r5f's library, codec PMC
set -u
O=gpurun_out
T=${1:-r5i}
mkdir -p $O/${T}_pmc
export TMPDIR=/tmp
bash scripts/gpu_round.sh $T tests || exit $?
for v in 0 d; do
  for b in 32 1; do
    if [ $v = d ]; then unset TTS_CODEC_X3P_ILV; else export TTS_CODEC_X3P_ILV=$v; fi
    timeout -k 10 120 python scripts/codec_probe32.py $b 650 >> $O/${T}_ab_codec_ilv.txt 2>&1 || exit $?
    echo "  (TTS_CODEC_X3P_ILV=$v)" >> $O/${T}_ab_codec_ilv.txt
  done
done
unset TTS_CODEC_X3P_ILV
cat $O/${T}_ab_codec_ilv.txt
export AB_V0=$PWD/ablib/lib_cur.so AB_V1=$PWD/tts-max_amd/tts_amd/libtts_mi355x.so
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_8.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/env_ab_probe.py TTS_LIB_PATH 32 1 > $O/${T}_ab_32.txt 2>&1 || exit $?
AB_ARCH=tts1-max timeout -k 10 400 python scripts/env_ab_probe.py TTS_LIB_PATH 8 1 > $O/${T}_ab_max8.txt 2>&1 || exit $?
cat $O/${T}_ab_8.txt $O/${T}_ab_32.txt $O/${T}_ab_max8.txt
unset AB_V0 AB_V1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d /tmp/${T}_codec1 -o pmc -- python3 scripts/codec_probe32.py 32 650 > $O/${T}_pmc/codec1.log 2>&1 || exit $?
python3 scripts/pmc_kernels.py "gemm_x3p_kernel<[^>]*>|gemm_bx3_kernel<[^>]*>|codec_attn_kernel<[^>]*>" /tmp/${T}_codec1 > $O/${T}_pmc/codec_pmc.json
cat $O/${T}_pmc/codec_pmc.json | grep -E "kernel|mfma_util|wait"
# where the codec pass's time goes: the x3p K loop's phases (stamps build) and the pass's idle time
TTS_LIB_PATH=$PWD/tts-max_amd/tts_amd/libtts_mi355x_stamps.so TTS_CODEC_STAMPS=1 timeout -k 10 120 \
  python scripts/codec_probe32.py 32 650 > $O/${T}_codec_stamps.txt 2>&1 || exit $?
cat $O/${T}_codec_stamps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/${T}_ctrace -o run -- \
  python3 scripts/codec_probe32.py 32 650 > $O/${T}_ctrace.log 2>&1 || exit $?
python3 scripts/trace_gaps.py $(find /tmp/${T}_ctrace -name "*kernel_trace.csv" | head -1) > $O/${T}_codec_gaps.txt
cat $O/${T}_codec_gaps.txt
