#!/bin/bash
# r5 ring-depth A/B: 17..32-row gate/up with a four-stage weight ring (TTS_RING4_32)
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_RING4_32 32 3 > gpurun_out/r5ring32_32.txt 2>&1 &&
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_RING4_32 24 2 > gpurun_out/r5ring32_24.txt 2>&1
