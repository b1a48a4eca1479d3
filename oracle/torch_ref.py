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


def frontend_port(raw, weights, params, n_fft=4096, hop=281):
    """The reference front end as BASELINE.md 3 specifies the CPU baseline:
    normalize (tfdataset.py:1916-1934) -> tf.signal.stft(pad_end) restated as
    torch.stft(center=False) on the end-padded clip with a periodic Hann window
    (:2026-2034) -> |X|^2 -> the DENSE batch_dot with the filterbank tiled over
    the batch (:2044-2051) -> PCEN + normalize_minmax (tfpcen.py).  raw [B, N]
    float32 -> [B, M, T] float32."""
    x = raw.to(torch.float32)
    x = x - x.amin(dim=-1, keepdim=True)
    x = x / x.amax(dim=-1, keepdim=True) + 1e-6
    x = (x - 0.5) * 2
    b, n = x.shape
    t = -(-n // hop)
    x = torch.nn.functional.pad(x, (0, (t - 1) * hop + n_fft - n))
    win = torch.hann_window(n_fft, periodic=True, dtype=torch.float32)
    spec = torch.stft(x, n_fft, hop, n_fft, win, center=False, return_complex=True)  # [B, F, T]
    power = spec.real ** 2 + spec.imag ** 2
    w = torch.as_tensor(weights, dtype=torch.float32)
    mel = torch.bmm(w.expand(b, -1, -1), power)                                        # [B, M, T]
    with torch.no_grad():
        return pcen_torch(mel.transpose(1, 2).contiguous(), params.to(torch.float32))
