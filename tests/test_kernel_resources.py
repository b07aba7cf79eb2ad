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
# the decode steps of the bench workloads and their neighbours, read from the engine's own step
# code in dry-run mode (tts_debug_step_plan): a new plan shape cannot escape the gate.
# (arch, decode rows): TTS-1 at configs[1]'s one row, configs[4]'s 8, configs[2]'s 32 and the
# row counts between / beyond them; TTS-1-Max at configs[3]'s 8 per GPU, 1 and 16
PLAN_CASES = [("tts1", r) for r in (1, 2, 4, 8, 12, 16, 17, 24, 32, 48, 64)] + \
             [("tts1-max", r) for r in (1, 8, 16, 32)]


def _hot_wgemm():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
    from tts_amd import configs
    from tts_amd.speechlm import step_plan

    hot = {}
    for arch, rows in PLAN_CASES:
        for k in step_plan(configs.LM_ARCHS[arch], rows):
            if k.startswith("wgemm_kernel<"):
                hot.setdefault(k[len("wgemm_kernel<"):-1], f"{arch} {rows} rows")
    return hot


UNITS = ["lm_gemm_store.hip", "lm_gemm_resid.hip", "lm_gemm_swiglu.hip", "lm_gemm_logits.hip", "lm_attn.hip",
         "lm_ops.hip", "lm_pgemm.hip", "codec_kernels.hip", "codec_gemm.hip", "lm_head_screen.hip"]

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


def test_step_plan_lists_the_bench_launches():
    """The dry run reproduces the launch structure the GPU runs: the one-row step is three
    launches a layer (QKV + attention + o_proj fused, gate/up, down) + the greedy head (int8
    screen + exact recompute of the units that can hold the argmax, lm_head_screen.hip) + finalize."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
    from tts_amd import configs
    from tts_amd.speechlm import step_plan

    one = step_plan(configs.LM_ARCHS["tts1"], 1)
    assert one[-2:] == ["head_screen_kernel<1, 32, 1, false>", "finalize_greedy_kernel"], one
    assert len([k for k in one if k.startswith("wgemm_kernel<")]) == 3, one
    assert "attn_decode_kernel<64>" not in one  # (fused into the QKV launch)
    b32 = step_plan(configs.LM_ARCHS["tts1"], 32)
    assert "attn_decode_kernel<64>" in b32 and "splitk_combine_norm" in b32, b32
    # 17..32 rows: the rows quantised once, then the screen with the int8 image alone in LDS
    assert b32[-3:] == ["head_rowquant_kernel", "head_screen_kernel<4, 32, 1, true>", "finalize_greedy_kernel"], b32
    # 2..16 rows: the attention and o_proj ride the QKV launch (its FROWS instantiation), the
    # RMSNorms run in the consumers' prologues, no standalone norm pass
    b8 = step_plan(configs.LM_ARCHS["tts1"], 8)
    assert "attn_decode_kernel<64>" not in b8 and "rmsnorm" not in b8, b8
    assert any(k.startswith("wgemm_kernel<8, 2, 1, 2, 4, 1, true, 2,") for k in b8), b8
    # 10..16 rows: the K-sliced down projection's combine normalises each row once for the next
    # QKV launch (TTS_NORM_ONCE 3), which then stages the rows without its RMSNorm prologue
    b16 = step_plan(configs.LM_ARCHS["tts1"], 16)
    assert "splitk_combine_norm" in b16 and "wgemm_kernel<16, 2, 1, 1, 16, 1, false, 0, 2, false, 16, true>" in b16, b16


def test_hot_wgemm_instantiations_do_not_spill(spills):
    hot = _hot_wgemm()
    assert len(hot) >= 10, hot
    found = {h: spills[_mangled(h)][1] for h in hot if _mangled(h) in spills}
    missing = {h: hot[h] for h in hot if h not in found}
    assert not missing, f"hot instantiations not compiled: {missing}"
    bad = {h: (n, hot[h]) for h, n in found.items() if n > 0}
    assert not bad, f"VGPR spills in hot-path GEMM instantiations: {bad}"


def test_attention_finalize_prefill_codec_kernels_do_not_spill(spills):
    bad = {k: n for k, (unit, n) in spills.items()
           if unit in ("lm_attn.hip", "lm_ops.hip", "lm_pgemm.hip", "codec_kernels.hip", "codec_gemm.hip",
                       "lm_head_screen.hip") and n > 0}
    assert not bad, f"VGPR spills: {bad}"
