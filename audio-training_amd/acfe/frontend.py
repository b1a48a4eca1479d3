"""Feature front end on the GPU: normalize, mix_up, STFT->mel, PCEN.

Mirrors the reference operators (tfdataset.normalize :1916-1934,
tfdataset.mix_up :930-955, tfdataset.raw_to_mel :2007-2059,
predict_utils.get_spect :163-239, tfpcen.PCEN :42-99) on torch device tensors,
executing the HIP kernels of csrc/frontend.hip through the C ABI.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import call, lib
from ._torch import dtype_code, ptr, require_cuda, stream

PAD_MODES = {"end": _lib.PAD_END, "constant": _lib.PAD_CENTER_CONSTANT, "reflect": _lib.PAD_CENTER_REFLECT}


def mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq) -> np.ndarray:
    """custommel.mel_f (custommel.py:18-54), computed by the C restatement in libacfe."""
    out = np.zeros((int(n_mels), 1 + int(n_fft) // 2), dtype=np.float32)
    call("acfe_mel_filterbank", int(sr), int(n_mels), float(fmin), float(fmax), int(n_fft), float(break_freq),
         out.ctypes.data_as(C.c_void_p))
    return out


class MelPlan:
    """Device plan (twiddles, window, banded filterbank) for one feature config.

    Equivalent of the reference's module globals MEL_WEIGHTS / NFFT /
    HOP_LENGTH set by tfdataset.get_dataset (tfdataset.py:430-460)."""

    def __init__(self, sr=48000, n_fft=4096, hop=281, n_mels=128, fmin=100, fmax=11000, break_freq=1000,
                 weights: np.ndarray | None = None, device=None):
        self.sr, self.n_fft, self.hop, self.n_mels = int(sr), int(n_fft), int(hop), int(n_mels)
        self.fmin, self.fmax, self.break_freq = fmin, fmax, break_freq
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if weights is None:
            weights = mel_filterbank(sr, n_mels, fmin, fmax, n_fft, break_freq)
        self.weights = np.ascontiguousarray(weights, dtype=np.float32)
        if self.weights.shape != (self.n_mels, 1 + self.n_fft // 2):
            raise ValueError(f"weights shape {self.weights.shape} does not match n_mels/n_fft")
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            call("acfe_plan_create", self.sr, self.n_fft, self.hop, self.n_mels, float(fmin), float(fmax),
                 float(break_freq), self.weights.ctypes.data_as(C.c_void_p), C.byref(h))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        # at interpreter shutdown the module globals may already be gone
        if h is not None and h.value and lib is not None:
            lib.acfe_plan_destroy(h)
            self._h = None

    def num_frames(self, n_samples: int, pad_mode: str = "end") -> int:
        return call("acfe_plan_num_frames", self._h, int(n_samples), PAD_MODES[pad_mode])

    def mel(self, raw: torch.Tensor, stats: torch.Tensor | None = None, pad_mode="end", power=2,
            layout="btm", n: int | None = None, clip_stride: int | None = None, batch: int | None = None,
            out: torch.Tensor | None = None, timer: list | None = None) -> torch.Tensor:
        """raw [B, N] fp32 (or a 1-D recording with explicit n / clip_stride / batch
        for overlapping windows) -> mel [B,T,M] ("btm") or [B,M,T] ("bmt")."""
        require_cuda(raw, stats)
        if raw.dtype != torch.float32:
            raise TypeError("raw audio must be float32")
        if raw.dim() == 2 and n is None:
            batch, n, clip_stride = raw.shape[0], raw.shape[1], raw.shape[1]
        if n is None or clip_stride is None or batch is None:
            raise ValueError("1-D input needs n, clip_stride and batch")
        if raw.numel() < (batch - 1) * clip_stride + n:
            raise ValueError("raw buffer too small for batch/clip_stride/n")
        t = self.num_frames(n, pad_mode)
        shape = (batch, t, self.n_mels) if layout == "btm" else (batch, self.n_mels, t)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=raw.device)
        elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("bad out tensor")
        e0 = None
        if timer is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        call("acfe_mel_fwd", self._h, ptr(raw), int(clip_stride), int(batch), int(n), ptr(stats),
             PAD_MODES[pad_mode], int(power), ptr(out), _lib.LAYOUT_BTM if layout == "btm" else _lib.LAYOUT_BMT,
             stream())
        if timer is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            timer.append(("mel", e0, e1))
        return out


    def mel_from_spec(self, spec: torch.Tensor, power=1, layout="btm", out: torch.Tensor | None = None,
                      timer: list | None = None) -> torch.Tensor:
        """Stored magnitude spectrograms [B, F, T] fp32 (F = 1 + n_fft/2, the
        record's audio/spectogram reshaped (2049, 513), tfdataset.py:1082) ->
        mel = W . S^power [B,T,M] ("btm") or [B,M,T] ("bmt") (tfdataset.py:1089)."""
        require_cuda(spec)
        if spec.dtype != torch.float32 or spec.dim() != 3 or not spec.is_contiguous():
            raise TypeError("spectrograms must be contiguous float32 [B, F, T]")
        b, f, t = spec.shape
        if f != self.n_fft // 2 + 1:
            raise ValueError(f"expected {self.n_fft // 2 + 1} frequency bins, got {f}")
        shape = (b, t, self.n_mels) if layout == "btm" else (b, self.n_mels, t)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=spec.device)
        e0 = None
        if timer is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        call("acfe_mel_from_spec", self._h, ptr(spec), f * t, b, f, t, int(power), ptr(out),
             _lib.LAYOUT_BTM if layout == "btm" else _lib.LAYOUT_BMT, stream())
        if timer is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            timer.append(("mel", e0, e1))
        return out


def normalize_stats(x: torch.Tensor, n: int | None = None, clip_stride: int | None = None,
                    batch: int | None = None) -> torch.Tensor:
    """Per-clip {min, max(x-min)} (tfdataset.normalize reductions)."""
    require_cuda(x)
    if x.dim() == 2 and n is None:
        batch, n, clip_stride = x.shape[0], x.shape[1], x.shape[1]
    st = torch.empty((batch, 2), dtype=torch.float32, device=x.device)
    call("acfe_normalize_stats", ptr(x), int(clip_stride), int(batch), int(n), ptr(st), stream())
    return st


def normalize_apply(x: torch.Tensor, st: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """(x - min) / max(x - min) per clip with precomputed stats; [B, N] fp32."""
    require_cuda(x, st)
    y = torch.empty_like(x) if out is None else out
    call("acfe_normalize_apply", ptr(x), x.shape[1], x.shape[0], x.shape[1], ptr(st), ptr(y), stream())
    return y


def normalize(x: torch.Tensor) -> torch.Tensor:
    """tfdataset.normalize (tfdataset.py:1916-1934) on [B, N] fp32."""
    return normalize_apply(x, normalize_stats(x))


def mix_up(x1, x2, lam, stats1=None, stats2=None) -> torch.Tensor:
    """tfdataset.mix_up image blend (tfdataset.py:950); lam [B] fp32 on device."""
    require_cuda(x1, x2, lam, stats1, stats2)
    y = torch.empty_like(x1)
    call("acfe_mixup", ptr(x1), ptr(stats1), ptr(x2), ptr(stats2), ptr(lam), x1.shape[0], x1.shape[1], ptr(y),
         stream())
    return y


def sample_mixup_lambda(batch, alpha=0.5, chance=0.25, device=None) -> torch.Tensor:
    """tfdataset.sample_beta_distribution(batch, alpha, alpha) * 1[U < chance]
    (tfdataset.py:920-946); drawn on the host from torch's global generator."""
    gam = torch.distributions.Gamma(torch.tensor(float(alpha)), torch.tensor(1.0))
    g1, g2 = gam.sample((batch,)), gam.sample((batch,))
    lam = g1 / (g1 + g2)
    aug = (torch.rand(batch) < chance).float()
    return (lam * aug).to(torch.float32).to(device if device is not None else "cpu")


class _PCENFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mel_btm, params, eps, out_dtype, scope_minmax):
        require_cuda(mel_btm, params)
        b, t, m = mel_btm.shape
        dev = mel_btm.device
        npart = lib.acfe_pcen_partials(b, m)
        y = torch.empty((b, m, t), dtype=torch.float32, device=dev)
        part = torch.empty(2 * npart, dtype=torch.float32, device=dev)
        s = stream()
        call("acfe_pcen_fwd", ptr(mel_btm), b, t, m, ptr(params), float(eps), ptr(y), ptr(part), s)
        out = torch.empty((b, m, t), dtype=out_dtype, device=dev)
        stats = torch.empty(4, dtype=torch.float32, device=dev)
        call("acfe_pcen_normalize", ptr(y), y.numel(), ptr(part), npart, ptr(scope_minmax), ptr(out),
             dtype_code(out_dtype), ptr(stats), s)
        ctx.save_for_backward(mel_btm, params, stats)
        ctx.eps = eps
        return out

    @staticmethod
    def backward(ctx, dout):
        mel_btm, params, stats = ctx.saved_tensors
        b, t, m = mel_btm.shape
        dout = dout.contiguous()
        npart = lib.acfe_pcen_partials(b, m)
        ws = torch.empty(32 * npart, dtype=torch.float32, device=dout.device)
        dparams = torch.empty(4, dtype=torch.float32, device=dout.device)
        call("acfe_pcen_bwd", ptr(mel_btm), b, t, m, ptr(params), float(ctx.eps), ptr(stats), ptr(dout),
             dtype_code(dout.dtype), ptr(ws), ptr(dparams), stream())
        return None, dparams, None, None, None


def pcen(mel_btm: torch.Tensor, params: torch.Tensor, eps: float = 1e-6, out_dtype=torch.float32,
         scope_minmax: torch.Tensor | None = None) -> torch.Tensor:
    """tfpcen.PCEN.call + normalize_minmax: mel [B,T,M] -> normalised [B,M,T]."""
    return _PCENFunction.apply(mel_btm.contiguous(), params, eps, out_dtype, scope_minmax)


class PCEN(torch.nn.Module):
    """Trainable PCEN (tfpcen.py:42-99). Parameters packed as one device vector
    {gain 0.98, bias 2.0, root 2.0, smooth 0.04}; eps = 1e-6.  The unused
    `a-power` weight of the reference (tfpcen.py:78-86) is kept for checkpoint
    compatibility but does not enter the computation, as in the reference."""

    def __init__(self, gain=0.98, bias=2.0, root=2.0, smooth=0.04, eps=1e-6, out_dtype=torch.float32):
        super().__init__()
        self.params = torch.nn.Parameter(torch.tensor([gain, bias, root, smooth], dtype=torch.float32))
        self.a_power = torch.nn.Parameter(torch.tensor([-1.0]), requires_grad=False)
        self.eps = eps
        self.out_dtype = out_dtype

    def forward(self, mel_btm, scope_minmax=None):
        return pcen(mel_btm, self.params, self.eps, self.out_dtype, scope_minmax)
