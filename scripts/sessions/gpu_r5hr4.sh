#!/bin/bash
# r5 lm_head ring-depth A/B (TTS_HEAD_RING4): 32 rows (=1), 8 rows (=2)
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_HEAD_RING4 32 3 > gpurun_out/r5hr4_32.txt 2>&1 &&
AB_V1=2 timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_HEAD_RING4 8 2 > gpurun_out/r5hr4_8.txt 2>&1
