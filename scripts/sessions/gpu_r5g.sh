#!/bin/bash
# round 5, session g: PMC diagnostics of the codec GEMM (gemm_x3p, 32 x 650 codes) and of the
# bs=32 prefill GEMMs (MFMA busy); bs=32 A/B of o_proj unsliced (no combine launch) with the
# gate/up RMSNorm in its LDS prologue
set -u
O=gpurun_out
T=${1:-r5g}
mkdir -p $O/${T}_pmc
export TMPDIR=/tmp
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d /tmp/${T}_codec$i -o pmc -- \
    python3 scripts/codec_probe32.py 32 650 > $O/${T}_pmc/codec$i.log 2>&1 || exit $?
done
python3 scripts/pmc_kernels.py "gemm_x3p_kernel<[^>]*>|gemm_bx3_kernel<[^>]*>|codec_attn_kernel<[^>]*>" /tmp/${T}_codec1 /tmp/${T}_codec2 \
  /tmp/${T}_codec3 /tmp/${T}_codec4 > $O/${T}_pmc/codec_pmc.json
cat $O/${T}_pmc/codec_pmc.json | head -80
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/${T}_prefill -o pmc -- \
  python3 bench.py --batch 32 --steps 1 --warmup 0 --new 8 --no-cpu-baseline --no-secondary --kernel-iters 1 \
  > $O/${T}_pmc/prefill.log 2>&1 || exit $?
python3 scripts/pmc_kernels.py "pgemm_kernel<[^>]*>|attn_prefill_kernel<[^>]*>" /tmp/${T}_prefill > $O/${T}_pmc/prefill_pmc.json
cat $O/${T}_pmc/prefill_pmc.json
export AB_V0=1 AB_V1=0
TTS_NORM32=1 timeout -k 10 400 python scripts/env_ab_probe.py TTS_KSLICE32_RESID 32 2 > $O/${T}_ab_oproj32_norm32.txt 2>&1 || exit $?
timeout -k 10 400 python scripts/env_ab_probe.py TTS_KSLICE32_RESID 32 1 > $O/${T}_ab_oproj32.txt 2>&1
rc=$?
cat $O/${T}_ab_oproj32_norm32.txt $O/${T}_ab_oproj32.txt
exit $rc
