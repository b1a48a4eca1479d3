"""Small helpers shared by the torch-facing wrappers."""
from __future__ import annotations

import torch

from ._lib import DTYPE_BF16, DTYPE_F32


def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DTYPE_F32
    if dt == torch.bfloat16:
        return DTYPE_BF16
    raise TypeError(f"unsupported dtype {dt}")


def require_cuda(*ts: torch.Tensor):
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("acfe ops take contiguous device tensors")
