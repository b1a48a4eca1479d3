"""ctypes binding of libacfe.so (the C ABI declared in include/acfe.h).

There is no fallback: if the HIP library is missing or fails to load, importing
this module raises.  Build it with `make -C audio-training_amd/csrc` (or
`__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# ACFE_LIB: an alternative build of the same library (A/B experiments, tools/ab_lib.sh)
LIB_PATH = Path(os.environ.get("ACFE_LIB") or Path(__file__).resolve().parent / "libacfe.so")

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float
F64 = C.c_double

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES: dict[str, list] = {
    "acfe_version": [],
    "acfe_last_error": [],
    "acfe_crc32c": [P, C.c_size_t, C.c_uint32],
    "acfe_tfr_open": [C.c_char_p, I32, P],
    "acfe_tfr_next": [P, I32, P, P],
    "acfe_tfr_close": [P],
    "acfe_example_audio": [P, C.c_uint64, C.c_char_p, P, I64, P, I32, P],
    "acfe_mel_filterbank": [I32, I32, F64, F64, I32, F64, P],
    "acfe_plan_create": [I32, I32, I32, I32, F64, F64, F64, P, P],
    "acfe_plan_destroy": [P],
    "acfe_plan_num_frames": [P, I32, I32],
    "acfe_normalize_stats": [P, I64, I32, I32, P, P],
    "acfe_normalize_apply": [P, I64, I32, I32, P, P, P],
    "acfe_mixup": [P, P, P, P, P, I32, I32, P, P],
    "acfe_copy_rows": [P, I64, I64, P, P, I64, I64, P, I32, I32, P],
    "acfe_mel_fwd": [P, P, I64, I32, I32, P, I32, I32, P, I32, P],
    "acfe_mel_from_spec": [P, P, I64, I32, I32, I32, I32, P, I32, P],
    "acfe_pcen_partials": [I32, I32],
    "acfe_pcen_fwd": [P, I32, I32, I32, P, F32, P, P, P],
    "acfe_pcen_normalize": [P, I64, P, I32, P, P, I32, P, P],
    "acfe_pcen_bwd": [P, I32, I32, I32, P, F32, P, P, I32, P, P, P],
    "acfe_conv2d_packed_shape": [I32, I32, I32, I32, I32, I32, P, P],
    "acfe_conv2d_pack_weights": [P, I32, I32, I32, I32, I32, I32, P, P],
    "acfe_conv2d_pack_weights_batch": [P, I32, I64, I32, P],
    "acfe_conv2d_stats_rows": [I64, I32],
    "acfe_conv2d_fwd": [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, I32, P, P],
    "acfe_conv2d_fwd_dropout": [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, I32, P, F32,
                                C.c_uint64, P],
    "acfe_conv2d_dgrad": [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, I32, P, P],
    "acfe_conv2d_dgrad_workspace": [I32] * 13,
    "acfe_conv2d_dgrad_bn_rows": [I32] * 9,
    "acfe_conv2d_dgrad_bn": [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, I32, P, P, P, P, P,
                             I32, P, I32, P],
    "acfe_conv2d_wgrad_workspace": [I32, I32, I32, I32, I32, I32, I32, I32, I32],
    "acfe_conv2d_wgrad": [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, F32, I32, P, P],
    "acfe_conv_r64_enable": [I32],
    "acfe_mel_w5_frames": [I32],
    "acfe_conv2d_wgrad_bnbwd_rows": [I32] * 5,
    "acfe_conv2d_wgrad_bnbwd": [P, I32, I32, I32, I32, P, P, I32, P, P, I32, P, P, F32, C.c_uint64, P, P, F32, P, P,
                                P],
    "acfe_conv2d_dropout_keep_supported": [I32] * 6,
    "acfe_conv2d_fwd_dropout_keep": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, P, F32, C.c_uint64, P, P],
    "acfe_conv2d_fwd_bn_keep": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, P, F32, C.c_uint64, P, P, I32, P, P,
                                I32, P],
    "acfe_conv2d_wgrad_bnbwd_keep": [P, I32, I32, I32, I32, P, P, I32, P, P, I32, P, F32, C.c_uint64, P, P, P, F32,
                                     P, P, P],
    "acfe_stem_blocks": [I32, I32, I32],
    "acfe_stem_fold_weights": [P, I32, I32, I32, I32, P, P],
    "acfe_stem_fwd": [P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, P, I32, P, P],
    "acfe_stem_dgrad": [P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, I32, P],
    "acfe_stem_wgrad": [P, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, F32, P, P],
    "acfe_stem_bwd_bn": [P, P, P, I32, I32, I32, I32, I32, I32, I32, P, P, P, P, I32, P, I32, P, F32, P, P, P],
    "acfe_reduce_blocks": [I64],
    "acfe_bn_stats": [P, I64, I32, I32, P, P],
    "acfe_bn_finalize": [P, I32, I32, I32, F64, P, P, F32, F32, P, P, I32, P, P, P, P, P],
    "acfe_bn_apply": [P, I32, I64, I32, P, P, I32, P, I32, P],
    "acfe_bn_bwd_reduce": [P, I32, P, I32, I64, I32, P, P, P, P, I32, P, P],
    "acfe_bn_bwd_finalize": [P, I32, I32, F64, P, P, P, P, P, P, P],
    "acfe_bn_bwd_finalize_ex": [P, I32, I32, F64, P, P, P, P, P, P, I32, P],
    "acfe_bn_bwd_apply": [P, I32, P, I32, I64, I32, P, P, I32, P, P, P, I32, P],
    "acfe_bn_bwd_apply_dropout": [P, I32, P, I32, I64, I32, P, P, I32, P, F32, C.c_uint64, P, I32, P],
    "acfe_bn_bwd_apply_ex": [P, I32, P, I32, I64, I32, P, P, I32, P, P, F32, C.c_uint64, P, I32, P, P],
    "acfe_conv2d_pool_supported": [I32, I32, I32, I32, I32, I32, I32, I32],
    "acfe_conv2d_fwd_pool": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, P, F32, C.c_uint64, P, I32, P],
    "acfe_conv2d_dgrad_unpool": [P, P, I32, I32, I32, I32, P, I32, I32, I32, P, I32, P],
    "acfe_conv2d_wgrad_unpool": [P, I32, I32, I32, I32, P, P, I32, I32, I32, P, F32, I32, P, P],
    "acfe_bn_bwd_apply_pool": [P, I32, P, I32, I32, I32, I32, I32, P, P, I32, P, P, I32, P, I32, P, P],
    "acfe_bn_bwd_apply_sub": [P, I32, P, I32, I32, I32, I32, I32, P, P, I32, P, P, I32, P, I32, P, P],
    "acfe_conv2d_rows_supported": [I32, I32, I32, I32, I32, I32, I32, I32],
    "acfe_conv2d_fwd_add_supported": [I32, I32, I32, I32, I32, I32],
    "acfe_conv2d_fwd_add": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, I32, P, P, I32, P],
    "acfe_conv2d_bn_prologue_supported": [I32, I32, I32, I32, I32, I32],
    "acfe_conv2d_fwd_bn": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, P, F32, C.c_uint64, P, P, I32, P, I32, P],
    "acfe_conv2d_fwd_pool_bn": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, P, F32, C.c_uint64, P, P, P, I32, P,
                                I32, P],
    "acfe_conv2d_fwd_add_bn": [P, I32, I32, I32, I32, P, I32, I32, I32, P, P, I32, P, P, P, P, I32, P, I32, P],
    "acfe_c1bn_supported": [I32, I32],
    "acfe_c1bn_workspace": [I64, I32, I32],
    "acfe_c1bn_stats": [P, I64, I32, P, I32, P, P, P, P, P],
    "acfe_c1bn_apply": [P, I64, I32, P, I32, P, P, P, I32, P, P],
    "acfe_c1bn_bwd": [P, P, I64, I32, P, I32, P, P, P, P, P, I32, F64, P, P, P, P, P, P, P, P],
    "acfe_c1bn_stats_bn": [P, I64, I32, P, I32, P, P, P, P, P, P, I32, P],
    "acfe_c1bn_apply_bn": [P, I64, I32, P, I32, P, P, P, I32, P, P, P, I32, P],
    "acfe_c1bn_bwd_bn": [P, P, I64, I32, P, I32, P, P, P, P, P, I32, F64, P, P, P, P, P, P, P, P, P, I32, P],
    "acfe_channel_sum": [P, I64, I32, I32, P, P, F32, P],
    "acfe_add": [P, P, I64, I32, P, I32, P],
    "acfe_add_stats": [P, P, I64, I32, I32, P, I32, P, P],
    "acfe_relu_bwd_sum": [P, P, I64, I32, P, I32, P, P],
    "acfe_channel_sum_finalize": [P, I32, I32, F32, P, P],
    "acfe_relu_bwd": [P, P, I64, P, I32, P],
    "acfe_dropout": [P, I64, F32, C.c_uint64, P, I32, P],
    "acfe_cast": [P, I32, I64, P, I32, P],
    "acfe_sigmoid": [P, I64, P, P],
    "acfe_maxpool2d": [P, I32, I32, I32, I32, I32, I32, P, I32, P],
    "acfe_maxpool2d_bwd": [P, P, I32, I32, I32, I32, I32, I32, P, I32, P],
    "acfe_maxpool2d_fused": [P, I32, I32, I32, I32, I32, I32, P, P, F32, C.c_uint64, P, I32, P],
    "acfe_bn_maxpool2d_fused": [P, I32, I32, I32, I32, P, P, I32, I32, I32, P, P, P, I32, P],
    "acfe_maxpool2d_bwd_argmax": [P, P, I32, I32, I32, I32, I32, I32, F32, C.c_uint64, P, I32, P],
    "acfe_maxpool2d_bwd_argmax_bn": [P, P, I32, I32, I32, I32, I32, I32, P, I32, P, P, P, P, P, I32, P, P],
    "acfe_avgpool2d": [P, I32, I32, I32, I32, I32, P, I32, P],
    "acfe_avgpool2d_bwd": [P, I32, I32, I32, I32, I32, P, I32, P],
    "acfe_axis_pool": [P, I32, I64, I32, I32, F32, I32, P, P],
    "acfe_axis_pool_bwd": [P, I32, P, I64, I32, I32, F32, I32, P, P],
    "acfe_dense_fwd": [P, P, P, I32, I32, I32, P, P],
    "acfe_dense_bwd": [P, P, P, I32, I32, I32, P, P, P, P],
    "acfe_loss": [P, P, I32, I32, I32, F32, P, P, P, P],
    "acfe_adam_step": [P, P, P, P, I64, F32, F32, F32, F32, F32, P],
}
_RESTYPES = {"acfe_last_error": C.c_char_p, "acfe_conv2d_wgrad_workspace": I64, "acfe_conv2d_dgrad_workspace": I64, "acfe_crc32c": C.c_uint32,
             "acfe_c1bn_workspace": I64}

PAD_END, PAD_CENTER_CONSTANT, PAD_CENTER_REFLECT = 0, 1, 2
LAYOUT_BTM, LAYOUT_BMT = 0, 1
DTYPE_F32, DTYPE_BF16 = 0, 1
E_INVAL = -1000
E_IO, E_CORRUPT = -1002, -1003


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
