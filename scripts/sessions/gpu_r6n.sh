#!/bin/bash
# round-6 final measurement, part 2 (gpu_r6h.sh: the TTS-1-Max configs[3] shard line + stats,
# PMC HBM traffic of the bench kernels, the RCCL path at one rank), then the codec ring-depth
# A/B (gpu_r6o.sh)
set -u
bash scripts/sessions/gpu_r6h.sh r6n || exit $?
bash scripts/sessions/gpu_r6o.sh r6o || exit $?
echo done
