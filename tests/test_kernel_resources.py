"""Register spills are a build-time property: every kernel instantiation the decode step and the
codec launch must compile without VGPR spills (a spill is a scratch store per lane and wave, a
write stream to HBM the kernel's roofline does not have: round 4 found 11.4 MB of them per
launch in the 8-row TTS-1-Max QKV + attention + o_proj launch).

Compiles the kernel translation units for gfx950 with the compiler's resource remarks
(`-Rpass-analysis=kernel-resource-usage`, what scripts/kernel_resources.sh prints) and fails on
any spill in the hot-path instantiations: the ones rocprofv3 lists for the bench's bs=1, 8, 16,
32-row TTS-1 steps and the TTS-1-Max 8-row shard (profiles/*_kernel_stats.csv), plus every
kernel of the attention / finalize / codec units.  CPU only (hipcc cross-compiles)."""

import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tts-max_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# wgemm_kernel<WAVES, KU, MT_MAX, NG, KSPLIT, ASRC, NORM, EPI, R, EARLY, KSW, FROWS> launched by
# the decode steps of the bench workloads (TTS-1 1 / 8 / 16 / 32 rows, TTS-1-Max 8 rows)
HOT_WGEMM = [
    "8, 2, 2, 2, 4, 1, false, 2, 4, false, 4, false",     # gate/up 17..32 rows (four-stage ring)
    "16, 2, 1, 1, 16, 1, true, 0, 2, false, 16, true",    # QKV + attention (+ o_proj), 2..16 rows, TTS-1
    "8, 2, 2, 1, 16, 1, false, 0, 2, false, 4, false",    # K-sliced qkv / o_proj, 17..32 rows
    "16, 4, 2, 1, 16, 1, false, 0, 1, false, 16, false",  # down K chunks, 17..32 rows
    "8, 2, 1, 2, 4, 1, true, 2, 4, false, 4, false",      # gate/up 4..16 rows (four-stage ring)
    "4, 8, 2, 1, 1, 1, false, 3, 2, false, 1, false",     # lm_head 17..32 rows
    "16, 4, 1, 1, 16, 1, false, 1, 2, false, 16, false",  # down 2..16 rows
    "8, 2, 1, 2, 4, 1, true, 2, 2, true, 4, false",       # gate/up one row
    "16, 2, 1, 1, 16, 1, true, 0, 2, true, 16, false",    # QKV + attention + o_proj one row
    "4, 8, 1, 1, 1, 1, true, 3, 2, false, 1, false",      # lm_head 2..16 rows
    "16, 4, 1, 1, 16, 1, false, 1, 2, true, 16, false",   # down one row
    "4, 8, 1, 1, 1, 1, true, 3, 2, true, 1, false",       # lm_head one row
    "16, 2, 1, 1, 16, 1, false, 1, 2, true, 16, false",   # o_proj one row (separate launch)
    "16, 4, 1, 1, 16, 1, true, 0, 2, false, 16, true",    # TTS-1-Max QKV + attention + o_proj, 8 rows
    "16, 4, 1, 1, 16, 0, false, 1, 1, false, 16, false",  # TTS-1-Max down (A fragments from L2), 8 rows
    "16, 4, 1, 1, 16, 1, true, 0, 2, false, 16, false",   # TTS-1-Max QKV (separate launch), 8 rows
]
UNITS = ["lm_gemm_store.hip", "lm_gemm_resid.hip", "lm_gemm_swiglu.hip", "lm_gemm_logits.hip", "lm_attn.hip",
         "lm_ops.hip", "codec_kernels.hip", "codec_gemm.hip"]

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


def _remarks(unit):
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "--cuda-device-only", "-c",
           os.path.join(CSRC, unit), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out, name = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"remark:\s+VGPRs Spill: (\d+)", line)
        if m and name:
            out[name] = int(m.group(1))
    return out


def _mangled(args):
    """Itanium mangling of tts::wgemm_kernel<...>(tts::WgemmArgs) for the template arguments."""
    parts = []
    for a in (x.strip() for x in args.split(",")):
        parts.append({"false": "Lb0E", "true": "Lb1E"}.get(a, f"Li{a}E"))
    return "_ZN3tts12wgemm_kernelI" + "".join(parts) + "EEvNS_9WgemmArgsE"


@pytest.fixture(scope="module")
def spills():
    with ThreadPoolExecutor(len(UNITS)) as ex:
        parts = list(ex.map(_remarks, UNITS))
    names = {}
    for unit, d in zip(UNITS, parts):
        for mangled, n in d.items():
            names[mangled] = (unit, n)
    return names


def test_hot_wgemm_instantiations_do_not_spill(spills):
    found = {h: spills[_mangled(h)][1] for h in HOT_WGEMM if _mangled(h) in spills}
    missing = [h for h in HOT_WGEMM if h not in found]
    assert not missing, f"hot instantiations not compiled: {missing}"
    bad = {h: n for h, n in found.items() if n > 0}
    assert not bad, f"VGPR spills in hot-path GEMM instantiations: {bad}"


def test_attention_finalize_codec_kernels_do_not_spill(spills):
    bad = {k: n for k, (unit, n) in spills.items() if unit in ("lm_attn.hip", "lm_ops.hip", "codec_kernels.hip", "codec_gemm.hip")
           and n > 0}
    assert not bad, f"VGPR spills: {bad}"
