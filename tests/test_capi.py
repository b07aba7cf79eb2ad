"""The C-ABI library loads and exports every symbol include/*.h declares (no compute)."""

import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("tts_mi355x.h", "tts_mi355x_ops.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(tts_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    from tts_amd import _lib

    lib = _lib.load_library()
    declared = _declared()
    assert declared, "no declarations parsed"
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_lib.EXPORTED_SYMBOLS) == declared


def test_abi_version_and_error_path():
    from tts_amd import _lib

    lib = _lib.load_library()
    assert lib.tts_abi_version() == 4
    # invalid argument path: no GPU work, error message set, status non-zero
    st = lib.tts_engine_create(0, None)
    assert st != 0
    assert b"null" in lib.tts_last_error()


def test_struct_layouts_match_header():
    from tts_amd import _lib

    # sizes follow the C declarations (all 4-byte fields except the uint64 seed / int64 shape)
    assert ctypes.sizeof(_lib.LmConfig) == 17 * 4
    assert ctypes.sizeof(_lib.GenParams) == 8 * 4 + 8 + 2 * 4  # + frequency_penalty, reserved (ABI 2)
    assert ctypes.sizeof(_lib.CodecConfig) == (4 + 8 + 5) * 4
    assert ctypes.sizeof(_lib.TensorDesc) == 8 + 8 + 4 + 4 + 32 + 8
