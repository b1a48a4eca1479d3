"""ctypes binding of libacfe.so (the C ABI declared in include/acfe.h).

There is no fallback: if the HIP library is missing or fails to load, importing
this module raises.  Build it with `make -C audio-training_amd/csrc` (or
`__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libacfe.so"

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float
F64 = C.c_double

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES: dict[str, list] = {
    "acfe_version": [],
    "acfe_last_error": [],
    "acfe_mel_filterbank": [I32, I32, F64, F64, I32, F64, P],
    "acfe_plan_create": [I32, I32, I32, I32, F64, F64, F64, P, P],
    "acfe_plan_destroy": [P],
    "acfe_plan_num_frames": [P, I32, I32],
    "acfe_normalize_stats": [P, I64, I32, I32, P, P],
    "acfe_normalize_apply": [P, I64, I32, I32, P, P, P],
    "acfe_mixup": [P, P, P, P, P, I32, I32, P, P],
    "acfe_mel_fwd": [P, P, I64, I32, I32, P, I32, I32, P, I32, P],
    "acfe_pcen_partials": [I32, I32],
    "acfe_pcen_fwd": [P, I32, I32, I32, P, F32, P, P, P],
    "acfe_pcen_normalize": [P, I64, P, I32, P, P, I32, P, P],
    "acfe_pcen_bwd": [P, I32, I32, I32, P, F32, P, P, I32, P, P, P],
}
_RESTYPES = {"acfe_last_error": C.c_char_p}

PAD_END, PAD_CENTER_CONSTANT, PAD_CENTER_REFLECT = 0, 1, 2
LAYOUT_BTM, LAYOUT_BMT = 0, 1
DTYPE_F32, DTYPE_BF16 = 0, 1
E_INVAL = -1000


class AcfeError(RuntimeError):
    pass


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: the HIP library must be built (make -C audio-training_amd/csrc); "
            "there is no CPU fallback for the acfe path"
        )
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, I32)
    return lib


lib = _load()


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        if rc == E_INVAL:
            raise AcfeError(f"{what}: invalid argument (ACFE_E_INVAL)")
        raise AcfeError(f"{what}: {lib.acfe_last_error().decode()} (rc={rc})")
    return rc


def call(name: str, *args) -> int:
    return check(getattr(lib, name)(*args), name)


def exported_symbols() -> list[str]:
    return list(SIGNATURES)
