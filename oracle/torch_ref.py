"""PyTorch-CPU restatements (ORACLE, test-only) of the differentiable parts of
the reference hot path, for gradient checks.  See oracle/__init__.py."""
from __future__ import annotations

import torch


def pcen_torch(mel_btm: torch.Tensor, params: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    """tfpcen.py:33-39 (EMA via sequential scan), :89-95 (PCEN.call),
    :105-110 (normalize_minmax).  mel [B,T,M] -> [B,M,T] (transposed to the
    model layout).  Differentiable w.r.t. params = {gain, bias, root, smooth};
    torch.amax/amin share the gradient equally among ties, like TF's
    reduce_max/reduce_min gradients."""
    gain = torch.minimum(params[0], torch.ones((), dtype=params.dtype))
    bias = params[1]
    root = torch.maximum(params[2], torch.ones((), dtype=params.dtype))
    w = torch.clamp(params[3], 0.0, 1.0)
    x = mel_btm.to(params.dtype)
    a = x[:, 0]
    outs = []
    for t in range(x.shape[1]):
        a = w * x[:, t] + (1.0 - w) * a
        outs.append(a)
    ema = torch.stack(outs, dim=1)
    inv_r = 1.0 / root
    y = (x / (eps + ema) ** gain + bias) ** inv_r - bias ** inv_r
    mx, mn = torch.amax(y), torch.amin(y)
    out = 2 * ((y - mn) / (mx - mn)) - 1
    return out.transpose(1, 2)
