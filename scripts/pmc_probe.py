"""Launch one decode-step kernel `iters` times (HBM-cold, rotating layers) so that a
`rocprofv3 --pmc ...` pass around this process measures its per-launch HBM traffic.
Used by bench.py (roofline.traffic); runnable by hand:

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o pmc -- \
        python3 scripts/pmc_probe.py --kernel gate_up --rows 1 --ctx 452 --iters 20
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))

import torch  # noqa: E402,F401  (share torch's HIP runtime)
from tts_amd import configs  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arch", default="tts1")
ap.add_argument("--kernel", default="gate_up")
ap.add_argument("--rows", type=int, default=1)
ap.add_argument("--ctx", type=int, default=452)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
m = MI355XSpeechLM.synthetic(configs.LM_ARCHS[args.arch], max_batch=max(args.rows, 1),
                             max_seq_len=args.ctx + 16)
ms, by = m.bench_kernel(args.kernel, rows=args.rows, ctx=args.ctx, iters=args.iters)
print(f"{args.kernel}: {ms * 1000:.2f} us/launch, {by:.0f} algorithmic bytes/launch", flush=True)
