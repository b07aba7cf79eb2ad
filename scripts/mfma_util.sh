#!/bin/bash
# MFMA utilisation of the codec's split-bf16 GEMM (gemm_bx3_kernel) and the prefill GEMM
# (pgemm_kernel) from one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE;
# MI355X_MICROARCH.md: MFMA busy counts cycles, GRBM_GUI_ACTIVE sums the 8 XCDs).
# usage (GPU box): [CODEC_B=32] scripts/mfma_util.sh   -> gpurun_out/pmc/mfma_util.json
# (the codec pass decodes CODEC_B utterances of 650 codes in one ragged batch)
set -u
OUT=gpurun_out/pmc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d /tmp/mfma_codec -o pmc -- python3 scripts/codec_probe32.py ${CODEC_B:-32} 650 > $OUT/mfma_codec.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d /tmp/mfma_prefill -o pmc -- python3 bench.py --batch 8 --steps 1 --warmup 0 --new 8 --no-cpu-baseline \
  --no-secondary --kernel-iters 1 > $OUT/mfma_prefill.log 2>&1 || exit $?
python3 scripts/mfma_parse.py /tmp/mfma_codec /tmp/mfma_prefill > $OUT/mfma_util.json
cat $OUT/mfma_util.json
