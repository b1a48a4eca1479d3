"""One data-parallel training step of the hot path, MI355X-native.

raw 3 s @ 48 kHz clips --(normalize, mix_up, normalize)--> STFT -> |X|^2 ->
mel (tfdataset.py:913-915, :474-481, :2007-2059) --> PCEN (tfpcen.py) -->
wr_resnet / wr_resnet_bird forward + backward --> loss (audiomodel.loss) -->
gradient all-reduce (RCCL, ~4 MB buckets of the flat gradient arena launched
during the backward as their gradients complete, acfe.dp.GradBuckets) -->
Adam (audiomodel.optimizer).  Every compute stage is a HIP kernel behind
include/acfe.h; torch provides memory, streams, autograd bookkeeping and
torch.distributed.
"""
from __future__ import annotations

import torch
from torch import nn

from . import dp
from . import frontend as fe
from . import ops
from .layers import Adam, ParamArena

allreduce_mean_ = dp.allreduce_mean_  # one-collective form (tests / callers of round 1)


class FrontEnd(nn.Module):
    """Device feature extractor: raw [B, N] fp32 -> model input [B, M, T] (dtype).

    With `pcen=True` the mel energies go through trainable PCEN +
    normalize_minmax (tfpcen.py:42-110); otherwise the mel power itself is
    the feature, as in the reference's raw_to_mel output (tfdataset.py:2049-2053)."""

    def __init__(self, n_mels=128, n_fft=4096, hop=281, sr=48000, fmin=100, fmax=11000, break_freq=1000,
                 pcen=True, dtype=torch.bfloat16, device=None, weights=None, power=2):
        super().__init__()
        # |X|^power of the raw-audio paths: 2 in raw_to_mel (tfdataset.py:2044) and
        # get_spect (predict_utils.py:215); 1 for a model trained on the stored
        # magnitude spectrograms (tfdataset.py:1085-1089), as its metadata records
        self.power = power
        self.plan = fe.MelPlan(sr, n_fft, hop, n_mels, fmin, fmax, break_freq, weights=weights, device=device)
        self.pcen = fe.PCEN(out_dtype=dtype) if pcen else None
        self.dtype = dtype
        self.timer = None  # bench.py: list receiving ("mel", ev0, ev1)

    def forward(self, x1, x2=None, lam=None, pad_mode="end", scope_minmax=None):
        st1 = fe.normalize_stats(x1)
        if x2 is not None:
            st2 = fe.normalize_stats(x2)
            src = fe.mix_up(x1, x2, lam, st1, st2)
            st = fe.normalize_stats(src)
        else:
            src, st = x1, st1
        # Normalise once into a scratch clip (frames overlap ~14.6x, so
        # normalising on load inside the STFT repeats the divide per frame).
        src = fe.normalize_apply(src, st, out=src if src is not x1 else None)
        if self.pcen is not None:
            mel = self.plan.mel(src, None, pad_mode=pad_mode, power=self.power, layout="btm", timer=self.timer)
            return self.pcen(mel, scope_minmax)
        mel = self.plan.mel(src, None, pad_mode=pad_mode, power=self.power, layout="bmt", timer=self.timer)
        return ops.cast(mel, self.dtype)


    def forward_spec(self, spec, scope_minmax=None):
        """Model input from stored magnitude spectrograms [B, F, T] (the
        load_raw=False records, tfdataset.py:1065-1102): banded mel of the
        magnitude (power 1), then PCEN when enabled, else the mel itself."""
        if self.pcen is not None:
            return self.pcen(self.plan.mel_from_spec(spec, power=1, layout="btm", timer=self.timer), scope_minmax)
        return ops.cast(self.plan.mel_from_spec(spec, power=1, layout="bmt", timer=self.timer), self.dtype)

    def forward_windows(self, rec, first, count, n=144000, hop=72000, pad_mode="constant", scope_minmax=None):
        """Features of `count` overlapping windows of one device recording `rec`
        (1-D fp32): window w covers rec[(first + w) * hop : ... + n].  The
        streaming predict path (predict_utils.load_samples :53-148 slides 3 s
        windows; here the windows are read in place via the clip stride)."""
        view = rec[first * hop:]
        st = fe.normalize_stats(view, n=n, clip_stride=hop, batch=count)
        if self.pcen is not None:
            mel = self.plan.mel(view, st, pad_mode=pad_mode, power=self.power, layout="btm", n=n, clip_stride=hop,
                                batch=count, timer=self.timer)
            return self.pcen(mel, scope_minmax)
        mel = self.plan.mel(view, st, pad_mode=pad_mode, power=self.power, layout="bmt", n=n, clip_stride=hop,
                            batch=count, timer=self.timer)
        return ops.cast(mel, self.dtype)


def mix_labels(y1: torch.Tensor, y2: torch.Tensor, lam: torch.Tensor, single_label=True) -> torch.Tensor:
    """Label half of tfdataset.mix_up (:946-954): hard lambda > 0.5 for single-label."""
    lw = (lam > 0.5).float() if single_label else lam
    lw = lw.reshape(-1, 1).to(y1.device)
    return y1 * lw + y2 * (1 - lw)


class Trainer:
    """Holds the front end, the model, one flat parameter arena for both, and
    Keras-Adam; `step` runs one full training iteration on device tensors."""

    def __init__(self, model: nn.Module, frontend: FrontEnd, lr=0.01, loss="cce", process_group=None,
                 device=None, bucket_bytes=dp.BUCKET_BYTES, pack_once=True):
        self.model, self.frontend, self.loss_mode = model, frontend, loss
        self.device = device or next(model.parameters()).device
        self.holder = nn.ModuleList([frontend, model])
        self.arena = ParamArena(self.holder, self.device)
        self.opt = Adam(self.arena, lr=lr)
        self.pg = process_group
        self.world = dp.world_size(process_group)
        self.packer = None  # ops.WeightPacker, built from the first step's packings
        self.pack_once = pack_once
        self.buckets = None
        if self.world > 1:
            self.buckets = dp.GradBuckets(self.arena.grad, self.arena.params, self.arena.offsets, bucket_bytes,
                                          process_group)
            # gradients autograd accumulates into the arena (stem, Dense, PCEN,
            # the 1x1+BN node) report through the post-accumulate hook; the
            # kernels that accumulate in place report via ops.grads_ready
            for p in self.arena.params:
                p.register_post_accumulate_grad_hook(self._grad_done)

    def _grad_done(self, p):
        if self.buckets is not None:
            self.buckets.ready(p)

    def train(self, mode=True):
        self.holder.train(mode)
        return self

    def step(self, x1, y, x2=None, lam=None):
        """One training iteration.  x1 [B, N] raw clips (x2 / lam: mix_up
        partner and weights), or [B, F, T] stored magnitude spectrograms (the
        load_raw=False path, no mix_up: tfdataset.py:503-504)."""
        # the conv weights change only in the Adam step: all their packed forms
        # for this step come from one launch (the first step records them)
        if self.packer is not None:
            ops._PACK_ACTIVE = self.packer.pack()
        elif self.pack_once:
            ops._PACK_LOG = []
        try:
            feats = self.frontend.forward_spec(x1) if x1.dim() == 3 else self.frontend(x1, x2, lam)
            z = self.model(feats)
            loss, dz = ops.loss_and_grad(z, y, self.loss_mode)
            self.arena.zero_grad()
            if self.buckets is None:
                z.backward(dz)
                scale = 1.0
            else:
                self.buckets.begin()
                ops.set_grad_ready(self.buckets.ready)
                try:
                    z.backward(dz)
                finally:
                    ops.set_grad_ready(None)
                scale = self.buckets.finish()
        finally:
            ops._PACK_ACTIVE = None
            log, ops._PACK_LOG = ops._PACK_LOG, None
        if self.packer is None and log and self.pack_once:
            # arena weights only (their storage is fixed); derived weights keep
            # the per-call packing
            arena_ptrs = {p.data_ptr() for p in self.arena.params}
            log = [e for e in log if e[0].data_ptr() in arena_ptrs]
            if log and len({d for _, d, _ in log}) == 1:
                try:
                    self.packer = ops.WeightPacker(log, self.device)
                except ValueError:  # beyond the batch kernel's 256 packings: keep per-call packing
                    self.pack_once = False
        self.opt.step(grad_scale=scale)
        return loss, z

    @torch.no_grad()
    def predict(self, x, pad_mode="end"):
        self.holder.eval()
        try:
            f = self.frontend.forward_spec(x) if x.dim() == 3 else self.frontend(x, pad_mode=pad_mode)
            return ops.sigmoid(self.model(f))
        finally:
            self.holder.train()
