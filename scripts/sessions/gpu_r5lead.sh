#!/bin/bash
# r5 lead combine (TTS_LEAD_COMBINE): o_proj's combine + RMSNorm as the leading workgroups of
# the 17..32-row gate/up launch.  A/B at 32 and 24 rows (ids md5 must match), then the batched
# GPU tests with it on
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_LEAD_COMBINE 32 3 > gpurun_out/r5lead_32.txt 2>&1 &&
timeout -k 10 300 python -u scripts/env_ab_probe.py TTS_LEAD_COMBINE 24 2 > gpurun_out/r5lead_24.txt 2>&1 &&
TTS_LEAD_COMBINE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "batch or chain or rows" > gpurun_out/r5lead_tests.log 2>&1
