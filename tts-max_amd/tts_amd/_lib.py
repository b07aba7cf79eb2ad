"""ctypes binding of libtts_mi355x.so (include/tts_mi355x.h, include/tts_mi355x_ops.h).

The shared library is built in-tree (``make -C tts-max_amd/csrc``) and is the only compute
path: there is no CPU fallback.  If the library is missing this module raises on import of
any engine object, so a GPU run can never silently test something else.

``torch`` is imported first on purpose: torch ships its own HIP runtime
(libamdhip64.so.7) and the library must bind to that same runtime instance (it resolves
by SONAME once torch has loaded it), otherwise device pointers and streams from torch
would belong to a second runtime.
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must load the HIP runtime before the library; see docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# TTS_LIB_PATH: load another build of the same library (A/B experiments, scripts/ab_*.sh)
LIB_PATH = os.environ.get("TTS_LIB_PATH") or os.path.join(_HERE, "libtts_mi355x.so")

TTS_OK = 0
DT_F32, DT_BF16, DT_F16, DT_I32, DT_I64 = 0, 1, 2, 3, 4
EPI_STORE, EPI_RESID, EPI_SWIGLU = 0, 1, 2

# Every symbol declared by include/tts_mi355x.h and include/tts_mi355x_ops.h.
EXPORTED_SYMBOLS = (
    "tts_abi_version",
    "tts_last_error",
    "tts_engine_create",
    "tts_engine_destroy",
    "tts_lm_load",
    "tts_generate",
    "tts_generate_begin",
    "tts_generate_continue",
    "tts_generate_read",
    "tts_slots_open",
    "tts_slots_add",
    "tts_slots_add_seeded",
    "tts_slots_step",
    "tts_slots_read",
    "tts_slots_release",
    "tts_lm_score",
    "tts_lm_score_decode",
    "tts_lm_id_to_code",
    "tts_lm_last_timing",
    "tts_lm_bench_kernel",
    "tts_codec_load",
    "tts_codec_decode",
    "tts_codec_samples_per_code",
    "tts_encoder_load",
    "tts_encoder_encode",
    "tts_encoder_encode_features",
    "tts_synth_fill",
    "tts_op_retile",
    "tts_op_wgemm",
    "tts_debug_step_plan",
    "tts_op_pgemm",
    "tts_op_sample",
    "tts_op_rmsnorm",
    "tts_op_gemm_f32",
)


class TensorDesc(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char_p),
        ("data", ctypes.c_void_p),
        ("dtype", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("shape", ctypes.c_int64 * 4),
        ("on_device", ctypes.c_int32),
    ]


class LmConfig(ctypes.Structure):
    _fields_ = [
        ("hidden_size", ctypes.c_int32),
        ("num_layers", ctypes.c_int32),
        ("num_heads", ctypes.c_int32),
        ("num_kv_heads", ctypes.c_int32),
        ("head_dim", ctypes.c_int32),
        ("intermediate_size", ctypes.c_int32),
        ("vocab_size", ctypes.c_int32),
        ("tie_word_embeddings", ctypes.c_int32),
        ("rms_norm_eps", ctypes.c_float),
        ("rope_theta", ctypes.c_float),
        ("rope_llama3", ctypes.c_int32),
        ("rope_factor", ctypes.c_float),
        ("rope_low_freq_factor", ctypes.c_float),
        ("rope_high_freq_factor", ctypes.c_float),
        ("rope_original_max_position", ctypes.c_int32),
        ("max_batch", ctypes.c_int32),
        ("max_seq_len", ctypes.c_int32),
    ]


class GenParams(ctypes.Structure):
    _fields_ = [
        ("max_length", ctypes.c_int32),
        ("min_new_tokens", ctypes.c_int32),
        ("eos_token_id", ctypes.c_int32),
        ("do_sample", ctypes.c_int32),
        ("repetition_penalty", ctypes.c_float),
        ("temperature", ctypes.c_float),
        ("top_p", ctypes.c_float),
        ("top_k", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("frequency_penalty", ctypes.c_float),
        ("reserved", ctypes.c_int32),
    ]


class CodecConfig(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32),
        ("token_rate", ctypes.c_int32),
        ("hop_length", ctypes.c_int32),
        ("n_upsample", ctypes.c_int32),
        ("upsample_factors", ctypes.c_int32 * 4),
        ("kernel_sizes", ctypes.c_int32 * 4),
        ("hidden_dim", ctypes.c_int32),
        ("depth", ctypes.c_int32),
        ("heads", ctypes.c_int32),
        ("vq_dim", ctypes.c_int32),
        ("max_codes", ctypes.c_int32),
    ]


class TtsError(RuntimeError):
    """A non-zero tts_status from the library."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"tts status {status}: {msg}")
        self.status = status


_lib = None


def load_library() -> ctypes.CDLL:
    """Loads (once) and returns the library; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `make -C tts-max_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH)
    P, I32, I64, U64, F32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    pi32 = ctypes.POINTER(ctypes.c_int32)
    sig = {
        "tts_abi_version": (I32, []),
        "tts_last_error": (ctypes.c_char_p, []),
        "tts_engine_create": (I32, [I32, ctypes.POINTER(P)]),
        "tts_engine_destroy": (None, [P]),
        "tts_lm_load": (I32, [P, ctypes.POINTER(LmConfig), ctypes.POINTER(TensorDesc), I32]),
        "tts_generate": (I32, [P, ctypes.POINTER(GenParams), pi32, pi32, I32, pi32, I32, pi32, P]),
        "tts_generate_begin": (I32, [P, ctypes.POINTER(GenParams), pi32, pi32, I32, P]),
        "tts_generate_continue": (I32, [P, I32, pi32]),
        "tts_generate_read": (I32, [P, pi32, I32, pi32]),
        "tts_slots_open": (I32, [P, ctypes.POINTER(GenParams), I32, P]),
        "tts_slots_add": (I32, [P, I32, pi32, I32, I32]),
        "tts_slots_add_seeded": (I32, [P, I32, pi32, I32, I32, ctypes.c_uint64]),
        "tts_slots_step": (I32, [P, I32, pi32]),
        "tts_slots_read": (I32, [P, I32, pi32, I32, pi32, pi32]),
        "tts_slots_release": (I32, [P, I32]),
        "tts_lm_score": (I32, [P, pi32, pi32, I32, I32, ctypes.POINTER(ctypes.c_float), P]),
        "tts_lm_score_decode": (I32, [P, pi32, pi32, I32, I32, pi32, I32, ctypes.POINTER(ctypes.c_float), P]),
        "tts_lm_id_to_code": (I32, [P, pi32, I32, pi32]),
        "tts_lm_last_timing": (I32, [P, ctypes.POINTER(F32), ctypes.POINTER(F32), pi32]),
        "tts_lm_bench_kernel": (I32, [P, I32, I32, I32, I32, ctypes.POINTER(F32), ctypes.POINTER(ctypes.c_double)]),
        "tts_codec_load": (I32, [P, ctypes.POINTER(CodecConfig), ctypes.POINTER(TensorDesc), I32]),
        "tts_codec_decode": (I32, [P, pi32, pi32, I32, P, I32, ctypes.POINTER(ctypes.c_int64), P]),
        "tts_codec_samples_per_code": (I32, [P, pi32]),
        "tts_encoder_load": (I32, [P, P, I32]),
        "tts_encoder_encode": (I32, [P, ctypes.POINTER(F32), ctypes.c_int64, ctypes.POINTER(F32), I32, pi32, I32,
                                     pi32, ctypes.POINTER(F32)]),
        "tts_encoder_encode_features": (I32, [P, ctypes.POINTER(F32), ctypes.c_int64, ctypes.POINTER(F32), I32,
                                              pi32, I32, pi32, ctypes.POINTER(F32)]),
        "tts_synth_fill": (I32, [P, I32, I64, U64, F32, P]),
        "tts_op_retile": (I32, [P, P, I32, I32, I32, P]),
        "tts_op_wgemm": (I32, [P, I32, I32, I32, P, I32, P, F32, P, I32, P, I32, P]),
        "tts_op_pgemm": (I32, [P, I32, I32, P, I32, P, I32, P, I32, P]),
        "tts_op_sample": (I32, [P, I32, I32, F32, I32, F32, ctypes.c_uint64, I32, P, I32, P, P, P]),
        "tts_op_rmsnorm": (I32, [P, P, F32, P, I32, I32, P]),
        "tts_op_gemm_f32": (I32, [P, I32, I32, I32, P, I32, P, P, I32, P, I32, P]),
        "tts_debug_step_plan": (I32, [ctypes.POINTER(LmConfig), I32, I32, ctypes.c_char_p, I32]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("TTS_LIB_PATH") and not hasattr(lib, name):
            continue  # A/B runs against an older build (scripts/ab_bench.sh): its ABI subset
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int) -> None:
    if status != TTS_OK:
        msg = load_library().tts_last_error().decode(errors="replace")
        raise TtsError(status, msg)


def torch_dtype_code(t: torch.Tensor) -> int:
    return {torch.float32: DT_F32, torch.bfloat16: DT_BF16, torch.float16: DT_F16,
            torch.int32: DT_I32, torch.int64: DT_I64}[t.dtype]


def make_descs(tensors: dict[str, torch.Tensor]):
    """Builds a TensorDesc array for a name->tensor dict (tensors must stay alive)."""
    keep = []
    arr = (TensorDesc * len(tensors))()
    for i, (name, t) in enumerate(tensors.items()):
        t = t.contiguous()
        keep.append(t)
        nb = name.encode()
        keep.append(nb)
        arr[i].name = nb
        arr[i].data = t.data_ptr()
        arr[i].dtype = torch_dtype_code(t)
        arr[i].ndim = t.dim()
        for j, s in enumerate(t.shape):
            arr[i].shape[j] = s
        arr[i].on_device = 1 if t.is_cuda else 0
    return arr, keep


def stream_ptr(stream=None) -> int:
    """Raw hipStream_t of a torch stream (default: torch's current stream)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream
