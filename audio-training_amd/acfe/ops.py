"""Autograd operators over the acfe model kernels (csrc/conv.hip, csrc/nn.hip).

Every forward/backward here is one or more calls through the C ABI; torch is
used only for device memory (torch.empty), streams and autograd bookkeeping.
Layouts: activations NHWC (bf16 for training, fp32 for inference), weights
fp32 KRSC master copies packed to the compute dtype on every forward.
"""
from __future__ import annotations

import itertools
import os

import torch

from ._lib import call, lib
from ._torch import dtype_code, ptr, stream

F32, F64 = torch.float32, torch.float64

# ACFE_FUSE=0 runs the fused nodes (conv/pool + dropout + BN, Add + statistics,
# residual-gradient link) as their separate-op chains, for A/B checks.
FUSE = os.environ.get("ACFE_FUSE", "1") != "0"
# ACFE_UNPOOL=0: the pooled-conv node's backward materialises the 2x2 max-pool
# backward and runs the plain dgrad / wgrad instead of expanding it in their
# input staging (A/B switch).
UNPOOL = os.environ.get("ACFE_UNPOOL", "1") != "0"
# ACFE_BN_PROLOGUE=0: every BatchNormalization writes its output in its own
# apply pass instead of handing it to the consuming conv's input staging.
PROLOGUE = os.environ.get("ACFE_BN_PROLOGUE", "1") != "0"
# per-consumer switches of the prologue (A/B): the pooled 3x3 conv; the 1x1 + BN
# node (off by default: its four streaming passes each redo the BN of x, which
# measured 1 % slower per T1 step than the one apply pass it saves, r02ab)
PRO_POOL = os.environ.get("ACFE_BN_PROLOGUE_POOL", "1") != "0"
PRO_C1 = os.environ.get("ACFE_BN_PROLOGUE_C1", "0") != "0"
# ACFE_BN_PROLOGUE_1W=0: no BN prologue on the K = C = 128 one-wave conv (A/B)
PRO_1W = os.environ.get("ACFE_BN_PROLOGUE_1W", "1") != "0"
# ACFE_BN_REDUCE_FUSE=0: the BatchNormalization backward reduce runs as its own
# pass even where the kernel producing its gradient can form the sums (A/B)
FUSE_BN_REDUCE = FUSE and os.environ.get("ACFE_BN_REDUCE_FUSE", "1") != "0"
# ACFE_STEM_BN_FUSE=0: wr_resnet_bird's stem backward as separate BN apply,
# dgrad, wgrad and bias-sum passes instead of acfe_stem_bwd_bn (A/B)
STEM_BN_FUSE = os.environ.get("ACFE_STEM_BN_FUSE", "1") != "0"
# ACFE_BN_BWD_FUSE=0: the backward of Conv2D -> Dropout -> BatchNormalization
# runs the BN backward apply as its own pass instead of inside the conv's
# weight gradient (acfe_conv2d_wgrad_bnbwd) (A/B, tests)
FUSE_BN_BWD = FUSE and os.environ.get("ACFE_BN_BWD_FUSE", "1") != "0"
# ACFE_KEEP_BITS=0: the BN-fold weight gradient regenerates the dropout mask
# from the pair hashes instead of reading the forward's keep bits (A/B)
KEEP_BITS = os.environ.get("ACFE_KEEP_BITS", "1") != "0"
# ACFE_SUB_FUSE=0: a 1x1 "valid" stride-k conv shortcut hands its full-resolution
# dX (zero off the (k p, k q) pixels) to the BN backward instead of the P x Q
# values for acfe_bn_bwd_apply_sub (A/B, tests)
FUSE_SUB = FUSE and os.environ.get("ACFE_SUB_FUSE", "1") != "0"


def same_padding(n: int, k: int, s: int) -> tuple[int, int]:
    """TF/Keras padding="same": out = ceil(n/s), pad_before = total//2."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2


def valid_out(n: int, k: int, s: int) -> int:
    return (n - k) // s + 1


def _empty(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


def packed_shape(K, R, S, C, dt, flip):
    import ctypes as C_

    rp, cp = C_.c_int(), C_.c_int()
    call("acfe_conv2d_packed_shape", K, R, S, C, dt, flip, C_.byref(rp), C_.byref(cp))
    return rp.value, cp.value


# WeightPacker state: while a packer is active (inside Trainer.step) the packed
# forms it produced are returned instead of packing again; a list in
# _PACK_LOG records what a step packs (the packer is built from it)
_PACK_ACTIVE: dict | None = None
_PACK_LOG: list | None = None


def pack_weights(w: torch.Tensor, dtype: torch.dtype, flip: bool) -> torch.Tensor:
    K, R, S, C = w.shape
    dt = dtype_code(dtype)
    key = (w.data_ptr(), dt, int(flip))
    if _PACK_ACTIVE is not None:
        hit = _PACK_ACTIVE.get(key)
        if hit is not None:
            return hit
    if _PACK_LOG is not None:
        _PACK_LOG.append((w, dtype, bool(flip)))
    rp, cp = packed_shape(K, R, S, C, dt, int(flip))
    out = _empty((rp, cp), dtype, w.device)
    call("acfe_conv2d_pack_weights", ptr(w), K, R, S, C, dt, int(flip), ptr(out), stream())
    return out


class WeightPacker:
    """Every packed conv weight a training step uses, produced by ONE launch
    (acfe_conv2d_pack_weights_batch) at the start of the step instead of one
    acfe_conv2d_pack_weights launch per conv and orientation (52 per
    wr_resnet_bird step).  Built from the (weight, dtype, flip) list a step
    records in _PACK_LOG; the weights must keep their storage (arena views)."""

    def __init__(self, entries, device):
        import numpy as np

        seen, self.entries = set(), []
        for w, dtype, flip in entries:
            key = (w.data_ptr(), dtype_code(dtype), int(flip))
            if key not in seen:
                seen.add(key)
                self.entries.append((w, dtype, flip, key))
        dts = {dtype_code(d) for _, d, _, _ in self.entries}
        if len(dts) != 1 or not self.entries or len(self.entries) > 256:
            raise ValueError("WeightPacker: one dtype, 1..256 packings")
        self.dt = dts.pop()
        rec = np.zeros(len(self.entries), dtype=np.dtype(
            {"names": ["w", "out", "begin", "K", "R", "S", "C", "flip", "rows_p", "cols_p", "pad"],
             "formats": ["<u8", "<u8", "<i8"] + ["<i4"] * 8, "offsets": [0, 8, 16, 24, 28, 32, 36, 40, 44, 48, 52],
             "itemsize": 56}))
        self.out, total = {}, 0
        for i, (w, dtype, flip, key) in enumerate(self.entries):
            K, R, S, C = w.shape
            rp, cp = packed_shape(K, R, S, C, self.dt, int(flip))
            o = _empty((rp, cp), dtype, device)
            self.out[key] = o
            rec[i] = (w.data_ptr(), o.data_ptr(), total, K, R, S, C, int(flip), rp, cp, 0)
            total += rp * cp
        self.total = total
        self.table = torch.from_numpy(rec.view(np.uint8).copy()).to(device)

    def pack(self):
        call("acfe_conv2d_pack_weights_batch", ptr(self.table), len(self.entries), self.total, self.dt, stream())
        return self.out


def _no_stats(dev):
    return torch.empty(0, dtype=F64, device=dev)


# Live kernel timing for bench.py: weight data_ptr -> list of (kind, ev0, ev1).
# Events are recorded on the current torch stream, the stream every acfe
# kernel is launched on.
_WATCH: dict[int, list] = {}


def watch_conv(weight: torch.Tensor, store: list | None):
    if store is None:
        _WATCH.pop(weight.data_ptr(), None)
    else:
        _WATCH[weight.data_ptr()] = store


class _Timed:
    def __init__(self, w, kind):
        self.store = _WATCH.get(w.data_ptr()) if _WATCH else None
        self.kind = kind

    def __enter__(self):
        if self.store is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()

    def __exit__(self, *a):
        if self.store is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.store.append((self.kind, self.e0, e1))


# ------------------------------------------------------------------ conv
def keep_bits_ok(x, w, stride, pt, pl, P, Q, drop, want_stats) -> bool:
    """Can the dropout forward write its keep bits for the BN-fold weight
    gradient (acfe_conv2d_fwd_*_keep -> acfe_conv2d_wgrad_bnbwd_keep)?"""
    if not (KEEP_BITS and FUSE_BN_BWD and want_stats and drop is not None and drop[0] > 0.0
            and x.dtype == torch.bfloat16):
        return False
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    src = _pending(x)[0] if _pending(x) is not None else x  # (the BN input the prologue reads)
    return ((R, S, stride, pt, pl, P, Q) == (3, 3, 1, 1, 1, H, W) and src.is_contiguous()
            and src.data_ptr() % 16 == 0 and bool(lib.acfe_conv2d_dropout_keep_supported(N, H, W, C, K, 1)))


def _conv_fwd(x, w, b, stride, pt, pl, P, Q, want_stats, drop=None, keep=None):
    """acfe_conv2d_fwd[_dropout] -> (y, stats_partial); a pending BN output x
    (bn_prologue_ok's shapes) is convolved through the BN prologue.  keep: a
    uint8 [N, P, Q, K / 8] buffer for the dropout keep bits (keep_bits_ok)."""
    if _pending(x) is not None:
        if stride == 1 and (P, Q, pt, pl) == (x.shape[1], x.shape[2], 1, 1) and \
                bn_prologue_ok(x.shape, x.dtype, w):
            return _conv_fwd_bn(x, w, b, want_stats, drop, keep)
        materialize(x)
    N, H, W, C = x.shape
    K, R, S, Cw = w.shape
    assert Cw == C, (Cw, C)
    dt = dtype_code(x.dtype)
    wp = pack_weights(w, x.dtype, False)
    y = _empty((N, P, Q, K), x.dtype, x.device)
    stats = _no_stats(x.device)
    if want_stats:
        rows = lib.acfe_conv2d_stats_rows(N * P * Q, K)
        stats = _empty((rows, 2, wp.shape[0]), F64, x.device)
    args = (ptr(x), N, H, W, C, ptr(wp), K, R, S, stride, pt, pl, P, Q, ptr(b), ptr(y), dt,
            ptr(stats) if want_stats else None)
    with _Timed(w, "fwd"):
        if keep is not None:
            call("acfe_conv2d_fwd_dropout_keep", ptr(x), N, H, W, C, ptr(wp), K, pt, pl, ptr(b), ptr(y), ptr(stats),
                 float(drop[0]), int(drop[1]), ptr(keep), stream())
        elif drop is not None and drop[0] > 0.0:
            call("acfe_conv2d_fwd_dropout", *args, float(drop[0]), int(drop[1]), stream())
        else:
            call("acfe_conv2d_fwd", *args, stream())
    return y, stats


def direct_grad(p):
    """The flat-arena .grad view of parameter p when its gradient may be
    accumulated in place by the producing kernel (layers.ParamArena marks its
    parameters and zeroes the arena before each backward), else None."""
    if not getattr(p, "_acfe_arena", False):
        return None
    g = p.grad
    if g is None or g.dtype != F32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g


# Data-parallel overlap (acfe.dp.GradBuckets.ready): called with each arena
# parameter whose gradient a kernel has just finished accumulating in place
# (the kernel is enqueued on the current stream), so its bucket's all-reduce
# can start while the rest of the backward runs.  None outside a DP backward.
_GRAD_READY = None


def set_grad_ready(fn):
    global _GRAD_READY
    _GRAD_READY = fn


def grads_ready(*params):
    fn = _GRAD_READY
    if fn is not None:
        for p in params:
            if p is not None:
                fn(p)


def bn_src(x):
    """The BatchNormalization behind x (x = its output) when a dgrad of a conv
    reading x may form that BN's backward reduce (acfe_conv2d_dgrad_bn)."""
    return getattr(x, "_acfe_bn_src", None) if FUSE_BN_REDUCE else None


def _conv_bwd(x, w, dy, stride, pt, pl, P, Q, need_dx, need_dw, need_db, bias=None, bn=None):
    """dgrad / wgrad / bias gradient of _conv_fwd for the conv-output gradient dy.
    bn: bn_src(x) -- where acfe_conv2d_dgrad_bn covers the shape, dx comes back
    tagged with that BN's backward reduce slab (consumed by its _bn_bwd)."""
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    dt = dtype_code(x.dtype)
    dy = dy.contiguous()
    dx = dw = db = None
    s = stream()
    if need_dx:
        wf = pack_weights(w, x.dtype, True)
        dx = _empty(x.shape, x.dtype, x.device)
        ws = None
        brows = 0
        if bn is not None:
            xb = bn[0]
            brows = lib.acfe_conv2d_dgrad_bn_rows(N, H, W, C, K, R, S, stride, dt)
            if not (brows and xb.shape == x.shape and xb.dtype == x.dtype and xb.is_contiguous()
                    and xb.data_ptr() % 16 == 0 and P == H and Q == W):
                brows = 0
        if stride > 1:  # sub-pixel phases: packed sub-kernels + one phase image
            nb = lib.acfe_conv2d_dgrad_workspace(N, P, Q, K, C, R, S, stride, pt, pl, H, W, dt)
            ws = _empty((max(nb, 1),), torch.uint8, x.device)
        with _Timed(w, "dgrad"):
            if brows:
                xb, scale, shift, mean, invstd, brelu = bn
                part = _empty((brows, 2, C), F64, x.device)
                call("acfe_conv2d_dgrad_bn", ptr(dy), N, P, Q, K, ptr(wf), C, R, S, stride, pt, pl, H, W, ptr(dx), dt,
                     ptr(xb), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), int(brelu), ptr(part), brows, s)
                _tag(dx, "_acfe_bnpart", (part, brows, (xb.data_ptr(), tuple(xb.shape), brelu)))
            else:
                call("acfe_conv2d_dgrad", ptr(dy), N, P, Q, K, ptr(wf), C, R, S, stride, pt, pl, H, W, ptr(dx), dt,
                     ptr(ws), s)
    if need_dw:
        # arena parameters: the split-K combine accumulates straight into the
        # flat gradient buffer (beta 1) and autograd gets None -- no separate
        # add kernel per weight
        tgt = direct_grad(w)
        dw = tgt if tgt is not None else _empty(w.shape, F32, w.device)
        nws = lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, R, S, P, Q)
        ws = _empty((nws,), F32, x.device)
        with _Timed(w, "wgrad"):
            call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, R, S, stride, pt, pl, P, Q, ptr(dw),
                 1.0 if tgt is not None else 0.0, dt, ptr(ws), s)
        if tgt is not None:
            dw = None
            grads_ready(w)
    if need_db:
        tb = direct_grad(bias) if bias is not None else None
        db = channel_sum(dy, K, into=tb)
        if tb is not None:
            db = None
            grads_ready(bias)
    return dx, dw, db


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pt, pl, P, Q, want_stats, link=None):
        ctx.bias = b
        y, stats = _conv_fwd(x, w, b, stride, pt, pl, P, Q, want_stats)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pt, pl, P, Q, b is not None)
        ctx.bn = bn_src(x)
        ctx.link = link
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, w = ctx.saved_tensors
        stride, pt, pl, P, Q, has_b = ctx.conf
        need_dx = ctx.needs_input_grad[0] or ctx.link is not None
        N, H, W, C = x.shape
        K = w.shape[0]
        sub = (FUSE_SUB and ctx.link is not None and stride > 1 and w.shape[1] == 1 and w.shape[2] == 1
               and pt == 0 and pl == 0 and P == (H - 1) // stride + 1 and Q == (W - 1) // stride + 1
               and x.dtype == torch.bfloat16 and C % 8 == 0)
        if sub:
            # 1x1 "valid" stride-k shortcut: its dX is the 1x1 dgrad at the pixels
            # (k p, k q) only -- computed at P x Q (a stride-1 1x1 dgrad) and added
            # there by the BN's backward apply (acfe_bn_bwd_apply_sub)
            dyc = dy.contiguous()
            xs = x[:, ::stride, ::stride, :]
            dxc, dw, db = _conv_bwd(xs, w, dyc, 1, 0, 0, P, Q, True, False, has_b and ctx.needs_input_grad[2],
                                    bias=ctx.bias)
            if ctx.needs_input_grad[1]:
                _, dw, _ = _conv_bwd(x, w, dyc, stride, pt, pl, P, Q, False, True, False, bias=ctx.bias)
            ctx.link.sub = (dxc, stride)
            return None, dw, db, None, None, None, None, None, None, None
        dx, dw, db = _conv_bwd(x, w, dy, stride, pt, pl, P, Q, need_dx, ctx.needs_input_grad[1],
                               has_b and ctx.needs_input_grad[2], bias=ctx.bias, bn=ctx.bn)
        if ctx.link is not None:  # the BN reading x adds this gradient in its own backward
            ctx.link.grad = dx
            dx = None
        return dx, dw, db, None, None, None, None, None, None, None


def _sums_ok(t: torch.Tensor) -> bool:
    """Fused per-channel sums need C % 8 == 0, 256 % (C/8) == 0 and 16-B alignment."""
    C = t.shape[-1]
    return C % 8 == 0 and C <= 2048 and 256 % (C // 8) == 0 and t.data_ptr() % 16 == 0 and t.is_contiguous()


def _tag(t: torch.Tensor, name: str, value):
    """Attach a fact about a gradient tensor's CURRENT contents (its ReLU mask
    is applied, its channel sums are known).  Recorded with the tensor's
    version counter: if autograd later accumulates another gradient into it in
    place (InputBuffer add_), the version moves and the fact is dropped."""
    setattr(t, name, (value, t._version))


def _tagged(t: torch.Tensor, name: str):
    v = getattr(t, name, None)
    return v[0] if v is not None and v[1] == t._version else None


def _attach_sum(t: torch.Tensor, part: torch.Tensor, rows: int, nrows: int | None = None):
    """Finalize a fused channel-sum slab and cache it on the gradient tensor it
    sums, so the convolution receiving `t` as its output gradient takes its
    bias gradient from there instead of re-reading `t` (channel_sum)."""
    # finalized by channel_sum, possibly into an arena gradient; nrows: the
    # slab's row count when it is not acfe_reduce_blocks(rows) (a kernel's grid)
    _tag(t, "_acfe_chpart", (part, lib.acfe_reduce_blocks(rows) if nrows is None else nrows))


def channel_sum(x: torch.Tensor, C: int, into: torch.Tensor | None = None) -> torch.Tensor:
    """Per-channel sum of x [..., C] in fp32; with `into` (an arena gradient
    view) it is accumulated there instead (beta 1)."""
    out = into if into is not None else _empty((C,), F32, x.device)
    beta = 1.0 if into is not None else 0.0
    lazy = _tagged(x, "_acfe_chpart")
    if lazy is not None and lazy[0].shape[-1] == C:
        part, nrows = lazy
        call("acfe_channel_sum_finalize", ptr(part), nrows, C, beta, ptr(out), stream())
        return out
    rows = x.numel() // C
    part = _empty((lib.acfe_reduce_blocks(rows) * 2 * C,), F64, x.device)
    call("acfe_channel_sum", ptr(x), rows, C, dtype_code(x.dtype), ptr(part), ptr(out), beta, stream())
    return out


def conv2d(x, w, b=None, stride=1, padding="same", want_stats=False, link=None):
    """Keras Conv2D on NHWC x with KRSC weights. Returns (y, stats_partial).
    link: a ResidualLink of the BatchNormalization that also reads x (a
    residual block's conv shortcut): the backward hands dX to that BN, which
    adds it inside its own backward (with the ReLU mask of x when x is a ReLU
    output) instead of autograd accumulating it and a separate ReLU pass;
    the conv must then be created after the BN (its backward runs first)."""
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    if padding == "same":
        P, pt = same_padding(H, R, stride)
        Q, pl = same_padding(W, S, stride)
    elif padding == "valid":
        P, Q, pt, pl = valid_out(H, R, stride), valid_out(W, S, stride), 0, 0
    else:
        raise ValueError(padding)
    if link is not None and not (x.is_contiguous() and (P, Q) != (0, 0)):
        # the conv cannot hand dX over: autograd accumulates it instead, and
        # the linked BN must not wait for it (ResidualLink.declined)
        link.declined = True
        link = None
    return _Conv2dFn.apply(x, w, b, stride, pt, pl, P, Q, want_stats, link)


# ------------------------------------------------------------------ stem (folded C=1)
class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pt, pl, out_dtype, want_stats):
        # x: [N, H, W] (one folded channel); w: [16, R, S, Crep] fp32
        N, H, W = x.shape
        K, R, S, rep = w.shape
        weff = _empty((R, S, K), F32, x.device)  # folded, RSK
        s = stream()
        call("acfe_stem_fold_weights", ptr(w), K, R, S, rep, ptr(weff), s)
        y = _empty((N, H, W, K), out_dtype, x.device)
        stats = _no_stats(x.device)
        if want_stats:
            stats = _empty((lib.acfe_stem_blocks(N, H, W), 2, K), F64, x.device)
        call("acfe_stem_fwd", ptr(x), dtype_code(x.dtype), N, H, W, R, S, pt, pl, ptr(weff), ptr(b), ptr(y),
             dtype_code(out_dtype), ptr(stats) if want_stats else None, s)
        ctx.save_for_backward(x, w, weff)
        ctx.conf = (pt, pl, b is not None)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _ds):
        x, w, weff = ctx.saved_tensors
        pt, pl, has_b = ctx.conf
        N, H, W = x.shape
        K, R, S, rep = w.shape
        dy = dy.contiguous()
        s = stream()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _empty(x.shape, x.dtype, x.device)
            call("acfe_stem_dgrad", ptr(dy), dtype_code(dy.dtype), N, H, W, R, S, pt, pl, ptr(weff), ptr(dx),
                 dtype_code(x.dtype), s)
        if ctx.needs_input_grad[1]:
            dw = _empty(w.shape, F32, w.device)
            ws = _empty((lib.acfe_stem_blocks(N, H, W) * K * R * S,), F64, x.device)
            call("acfe_stem_wgrad", ptr(x), dtype_code(x.dtype), ptr(dy), dtype_code(dy.dtype), N, H, W, R, S, pt,
                 pl, rep, ptr(dw), 0.0, ptr(ws), s)
        if has_b and ctx.needs_input_grad[2]:
            db = channel_sum(dy, K)
        return dx, dw, db, None, None, None, None


class _StemBNPoolFn(torch.autograd.Function):
    """conv1_1 -> BatchNormalization -> MaxPool2D((kh, kw)) of wr_resnet_bird
    (wr_resnet_bird.py:22-30) as one node.  Forward: the _StemFn and _BNPoolFn
    kernels.  Backward: the pool backward forms the BN reduce slab
    (acfe_maxpool2d_bwd_argmax_bn) and acfe_stem_bwd_bn applies the BN backward
    while staging the stem's dgrad / wgrad / bias sums, so the BN input
    gradient is never stored (k_bn_bwd_apply8's 3 x 1.07 GB per T1 step)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, mmean, mvar, conf):
        pt, pl, out_dtype, kh, kw, relu, eps, momentum, want_stats = conf
        N, H, W = x.shape
        K, R, S, rep = w.shape
        dev = x.device
        s = stream()
        weff = _empty((R, S, K), F32, dev)
        call("acfe_stem_fold_weights", ptr(w), K, R, S, rep, ptr(weff), s)
        y = _empty((N, H, W, K), out_dtype, dev)
        st = _empty((lib.acfe_stem_blocks(N, H, W), 2, K), F64, dev)
        call("acfe_stem_fwd", ptr(x), dtype_code(x.dtype), N, H, W, R, S, pt, pl, ptr(weff), ptr(b), ptr(y),
             dtype_code(out_dtype), ptr(st), s)
        _, saved = _bn_fwd(y, gamma, beta, st, mmean, mvar, True, relu, eps, momentum, None)
        P, Q = H // kh, W // kw
        yp = _empty((N, P, Q, K), y.dtype, dev)
        amax = _empty((N, P, Q, K), torch.uint8, dev)
        pst = _no_stats(dev)
        if want_stats:
            pst = _empty((lib.acfe_reduce_blocks(N * P * Q), 2, K), F64, dev)
        call("acfe_bn_maxpool2d_fused", ptr(y), N, H, W, K, ptr(saved[0]), ptr(saved[1]), int(relu), kh, kw, ptr(yp),
             ptr(amax), ptr(pst) if want_stats else None, dtype_code(y.dtype), s)
        ctx.save_for_backward(x, w, weff, y, amax, *saved)
        ctx.conf, ctx.gb = conf, (gamma, beta)
        ctx.mark_non_differentiable(pst)
        return yp, pst

    @staticmethod
    def backward(ctx, g, _gs):
        x, w, weff, y, amax, *saved = ctx.saved_tensors
        pt, pl, out_dtype, kh, kw, relu, eps, momentum, want_stats = ctx.conf
        N, H, W, K = y.shape
        _, R, S, rep = w.shape
        dev = y.device
        s = stream()
        scale, shift, mean, invstd = saved
        g = g.contiguous()
        gu = _empty(y.shape, g.dtype, dev)
        rows = N * H * W
        nrows = lib.acfe_reduce_blocks(rows)
        part = _empty((nrows * 2 * K,), F64, dev)
        call("acfe_maxpool2d_bwd_argmax_bn", ptr(amax), ptr(g), N, H, W, K, kh, kw, ptr(gu), dtype_code(g.dtype),
             ptr(y), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), int(relu), ptr(part), s)
        coef, dgamma, dbeta = _bn_bwd_coef(part, nrows, K, rows, saved, True, ctx.gb, dev)
        nb = lib.acfe_stem_blocks(N, H, W)
        dx = _empty(x.shape, x.dtype, dev)
        dw = _empty(w.shape, F32, dev)
        ws = _empty((nb * K * R * S,), F64, dev)
        bp = _empty((nb, 2, K), F64, dev)
        call("acfe_stem_bwd_bn", ptr(gu), ptr(y), ptr(x), N, H, W, R, S, pt, pl, ptr(weff), ptr(scale), ptr(shift),
             ptr(coef), int(relu), ptr(dx), rep, ptr(dw), 0.0, ptr(bp), ptr(ws), s)
        db = None
        if ctx.needs_input_grad[2]:
            db = _empty((K,), F32, dev)
            call("acfe_channel_sum_finalize", ptr(bp), nb, K, 0.0, ptr(db), s)
        return (dx if ctx.needs_input_grad[0] else None), dw, db, dgamma, dbeta, None, None, None


def stem_bn_pool_ok(x, w, b, out_dtype, kh, kw) -> bool:
    """_StemBNPoolFn's shapes: training with autograd on, bf16 in and out, a
    bias, the 16-channel 5 x 5 / 3 x 3 stem and a fused pool shape."""
    K, R, S, _ = w.shape
    return (FUSE and FUSE_BN_REDUCE and STEM_BN_FUSE and torch.is_grad_enabled() and b is not None
            and x.dtype == torch.bfloat16 and out_dtype == torch.bfloat16 and x.dim() == 3 and x.is_contiguous()
            and K == 16 and R == S and R in (3, 5) and (kh, kw) in ((1, 2), (2, 2), (3, 3)))


def stem_bn_max_pool(x, w, b, out_dtype, gamma, beta, mmean, mvar, kh, kw, relu=False, eps=1e-3, momentum=0.99,
                     want_stats=False):
    """MaxPool2D((kh, kw))(BatchNormalization(stem_conv(x, w, b))) in training
    (stem_bn_pool_ok) -> (y, stats slab of y or None)."""
    N, H, W = x.shape
    _, R, S, _ = w.shape
    _, pt = same_padding(H, R, 1)
    _, pl = same_padding(W, S, 1)
    conf = (pt, pl, out_dtype, kh, kw, bool(relu), float(eps), float(momentum), bool(want_stats))
    y, st = _StemBNPoolFn.apply(x, w, b, gamma, beta, mmean, mvar, conf)
    return y, (st if want_stats else None)


def stem_conv(x, w, b, out_dtype, want_stats=False):
    """'same' stride-1 conv of a one-channel map x [N,H,W] whose Cin copies are folded."""
    N, H, W = x.shape
    _, R, S, _ = w.shape
    _, pt = same_padding(H, R, 1)
    _, pl = same_padding(W, S, 1)
    return _StemFn.apply(x, w, b, pt, pl, out_dtype, want_stats)


# ------------------------------------------------------------------ batch norm
class ResidualLink:
    """Hands the residual-branch gradient of an identity shortcut (ops.add) to
    the BatchNormalization that reads the same block input, so the two input
    gradients are summed inside acfe_bn_bwd_apply (its `add` operand) instead
    of by a separate autograd accumulation pass."""

    def __init__(self):
        self.grad = None
        self.pool = None  # (pooled gradient, k) from an avg_pool_same(x, k, link=...) shortcut
        # (dX at the pixels (k p, k q), k) from a 1x1 "valid" stride-k conv shortcut
        # (wr_resnet's transition blocks): its other pixels' gradient is zero
        self.sub = None
        # set by a consumer that could not take the link after all (ops.conv2d on a
        # non-contiguous x): its gradient reaches x through autograd instead
        self.declined = False

    @staticmethod
    def make():
        return ResidualLink() if FUSE else None

    def take(self):
        g, self.grad = self.grad, None
        return g

    def take_pool(self):
        p, self.pool = self.pool, None
        return p

    def take_sub(self):
        p, self.sub = self.sub, None
        return p


def _bn_fwd(x, gamma, beta, stats, mmean, mvar, training, relu, eps, momentum, out_dtype, defer=False, grad=False):
    """Batch statistics (given slab or acfe_bn_stats) -> finalize -> apply. Returns (y, saved).
    grad: a backward can run (the node's ctx.needs_input_grad); only then is y
    tagged with its BN input for a consumer dgrad's fused reduce.
    defer: y is returned unwritten, marked pending (x, scale, shift, relu); the
    consuming conv applies the BN in its input staging and fills y, or
    materialize(y) runs the apply pass."""
    C = x.shape[-1]
    rows = x.numel() // C
    dt = dtype_code(x.dtype)
    dev = x.device
    s = stream()
    scale, shift, mean, invstd = (_empty((C,), F32, dev) for _ in range(4))
    if training:
        if stats is None or stats.numel() == 0:
            nrows = lib.acfe_reduce_blocks(rows)
            part = _empty((nrows * 2 * C,), F64, dev)
            call("acfe_bn_stats", ptr(x), rows, C, dt, ptr(part), s)
            ld = C
        else:
            part = stats
            ld = stats.shape[-1]
            nrows = stats.numel() // (2 * ld)
        call("acfe_bn_finalize", ptr(part), nrows, ld, C, float(rows), ptr(gamma), ptr(beta), eps, momentum,
             ptr(mmean), ptr(mvar), 1, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), s)
    else:
        call("acfe_bn_finalize", None, 0, C, C, 0.0, ptr(gamma), ptr(beta), eps, momentum, ptr(mmean), ptr(mvar),
             0, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), s)
    if out_dtype is None:  # affine only: the caller applies it (bn_max_pool)
        return None, (scale, shift, mean, invstd)
    y = _empty(x.shape, out_dtype, dev)
    if FUSE_BN_REDUCE and training and grad:
        # a conv reading y may form this BN's backward reduce in its dgrad (_conv_bwd)
        y._acfe_bn_src = (x, scale, shift, mean, invstd, bool(relu))
    if defer and out_dtype == x.dtype:
        y._acfe_bn_pending = (x, scale, shift, bool(relu))
        return y, (scale, shift, mean, invstd)
    call("acfe_bn_apply", ptr(x), dt, rows, C, ptr(scale), ptr(shift), int(relu), ptr(y), dtype_code(out_dtype), s)
    return y, (scale, shift, mean, invstd)


# ------------------------------------------------------------------ BN prologue (deferred BN apply)
def bn_prologue_ok(x_shape, dtype, w) -> bool:
    """Can a conv with weights w [K][3][3][C] take its BN (+ReLU) input as a
    prologue (acfe_conv2d_fwd_bn / acfe_conv2d_fwd_add_bn)?"""
    if not (FUSE and PROLOGUE and dtype == torch.bfloat16 and len(x_shape) == 4):
        return False
    N, H, W, C = x_shape
    K, R, S, Cw = w.shape
    if K == 128 and not PRO_1W:
        return False
    return (R, S) == (3, 3) and Cw == C and bool(lib.acfe_conv2d_bn_prologue_supported(N, H, W, C, K, 1))


def _pending(t):
    return getattr(t, "_acfe_bn_pending", None)


def materialize(t: torch.Tensor) -> torch.Tensor:
    """Write a pending BN output with acfe_bn_apply (no-op for other tensors)."""
    p = _pending(t)
    if p is None:
        return t
    x, scale, shift, relu = p
    C = x.shape[-1]
    call("acfe_bn_apply", ptr(x), dtype_code(x.dtype), x.numel() // C, C, ptr(scale), ptr(shift), int(relu), ptr(t),
         dtype_code(t.dtype), stream())
    t._acfe_bn_pending = None
    return t


def _prologue_args(xb):
    """(BN input, scale, shift, relu) of the pending BN output xb, which the
    kernel about to run fills; xb stops being pending."""
    x, scale, shift, relu = _pending(xb)
    assert x.is_contiguous() and x.data_ptr() % 16 == 0 and xb.data_ptr() % 16 == 0
    xb._acfe_bn_pending = None
    return x, scale, shift, relu


def _conv_fwd_bn(xb, w, b, want_stats, drop, keep=None):
    """_conv_fwd of a pending BN output xb: acfe_conv2d_fwd_bn (3x3 "same" stride 1)."""
    N, H, W, C = xb.shape
    K = w.shape[0]
    x, scale, shift, relu = _prologue_args(xb)
    wp = pack_weights(w, xb.dtype, False)
    y = _empty((N, H, W, K), xb.dtype, xb.device)
    stats = _no_stats(xb.device)
    if want_stats:
        stats = _empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), F64, xb.device)
    rate, seed = drop if drop is not None and drop[0] > 0.0 else (0.0, 0)
    with _Timed(w, "fwd"):
        if keep is not None:
            call("acfe_conv2d_fwd_bn_keep", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(stats),
                 float(rate), int(seed), ptr(scale), ptr(shift), int(relu), ptr(xb), ptr(keep), dtype_code(xb.dtype),
                 stream())
        else:
            call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y),
                 ptr(stats) if want_stats else None, float(rate), int(seed), ptr(scale), ptr(shift), int(relu),
                 ptr(xb), dtype_code(xb.dtype), stream())
    return y, stats


def _bn_bwd_coef(part, prow, C, rows, saved, training, params, dev):
    """acfe_bn_bwd_finalize_ex over a reduce slab of prow rows -> (coef [3][C],
    dgamma, dbeta); arena parameters (gamma, beta): the finalizer accumulates
    into their gradient views and autograd gets None for them."""
    scale, shift, mean, invstd = saved
    tg = tb = None
    if params is not None:
        tg, tb = direct_grad(params[0]), direct_grad(params[1])
        if tg is None or tb is None:
            tg = tb = None
    dgamma = tg if tg is not None else _empty((C,), F32, dev)
    dbeta = tb if tb is not None else _empty((C,), F32, dev)
    coef = _empty((3 * C,), F32, dev)
    # eval mode: statistics are constants -> count -> inf removes the mean terms
    count = float(rows) if training else 1e300
    call("acfe_bn_bwd_finalize_ex", ptr(part), prow, C, count, ptr(scale), ptr(mean), ptr(invstd), ptr(dgamma),
         ptr(dbeta), ptr(coef), int(tg is not None), stream())
    if tg is not None:
        dgamma = dbeta = None
        grads_ready(*params)
    return coef, dgamma, dbeta


def _bn_bwd(x, dy, saved, relu, training, add=None, drop=None, mask_in=False, pool=None, params=None, part=None,
            sub=None):
    """(dx, dgamma, dbeta); dx += add; dx passed back through Dropout `drop` when given;
    mask_in: x is a ReLU output (ops.add), its backward [x > 0] is applied to dx here
    and dx is marked so that ops.add's backward skips its own pass.  part: the
    reduce slab [acfe_reduce_blocks(rows)][2][C] already formed by the kernel
    that produced dy (acfe_maxpool2d_bwd_argmax_bn): no reduce pass; the same
    when dy carries the slab of the dgrad that produced it (acfe_conv2d_dgrad_bn,
    tagged _acfe_bnpart for this x)."""
    scale, shift, mean, invstd = saved
    C = x.shape[-1]
    rows = x.numel() // C
    dev = x.device
    s = stream()
    nrows = lib.acfe_reduce_blocks(rows)
    prow = nrows
    if part is None:
        lazy = _tagged(dy, "_acfe_bnpart")
        if lazy is not None and lazy[2] == (x.data_ptr(), tuple(x.shape), bool(relu)):
            part, prow = lazy[0], lazy[1]
    dy = dy.contiguous()
    if part is None:
        part = _empty((nrows * 2 * C,), F64, dev)
        call("acfe_bn_bwd_reduce", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), rows, C, ptr(scale),
             ptr(shift), ptr(mean), ptr(invstd), int(relu), ptr(part), s)
    coef, dgamma, dbeta = _bn_bwd_coef(part, prow, C, rows, saved, training, params, dev)
    dx = _empty(x.shape, x.dtype, dev)
    rate, seed = drop if drop is not None and drop[0] > 0.0 else (0.0, 0)
    if add is not None:
        assert rate == 0.0
        add = add.contiguous()
        assert add.dtype == x.dtype and add.shape == x.shape
    # per-channel sums of dx ride along (bias gradient of the conv producing x)
    want_sum = FUSE and _sums_ok(dx) and _sums_ok(dy) and _sums_ok(x) and (add is None or _sums_ok(add))
    sums = _empty((nrows, 2, C), F64, dev) if want_sum else None
    flags = int(relu) | (2 if mask_in else 0)
    if sub is not None:  # 1x1 stride-k shortcut's dX (pixels (k p, k q) only) folded in
        gs, k = sub
        gs = gs.contiguous()
        assert rate == 0.0 and add is None and pool is None and gs.dtype == x.dtype
        N, H, W, _ = x.shape
        call("acfe_bn_bwd_apply_sub", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), N, H, W, C,
             ptr(scale), ptr(shift), flags, ptr(coef), ptr(gs), int(k), ptr(dx), dtype_code(x.dtype), ptr(sums), s)
        if want_sum:
            _attach_sum(dx, sums, rows)
        if mask_in:
            _tag(dx, "_acfe_relu_masked", True)
        return dx, dgamma, dbeta
    if pool is not None:  # shortcut AveragePooling2D(x) backward folded in
        gp, k = pool
        gp = gp.contiguous()
        assert rate == 0.0 and add is None and gp.dtype == x.dtype
        N, H, W, _ = x.shape
        call("acfe_bn_bwd_apply_pool", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), N, H, W, C,
             ptr(scale), ptr(shift), flags, ptr(coef), ptr(gp), int(k), ptr(dx), dtype_code(x.dtype), ptr(sums), s)
        if want_sum:
            _attach_sum(dx, sums, rows)
        if mask_in:
            _tag(dx, "_acfe_relu_masked", True)
        return dx, dgamma, dbeta
    call("acfe_bn_bwd_apply_ex", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), rows, C, ptr(scale),
         ptr(shift), flags, ptr(coef), ptr(add), float(rate), int(seed), ptr(dx), dtype_code(x.dtype), ptr(sums),
         s)
    if want_sum:
        _attach_sum(dx, sums, rows)
    if mask_in:
        _tag(dx, "_acfe_relu_masked", True)
    return dx, dgamma, dbeta


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, stats, mmean, mvar, training, relu, eps, momentum, out_dtype, link, defer):
        ctx.gb = (gamma, beta)
        y, saved = _bn_fwd(x, gamma, beta, stats, mmean, mvar, training, relu, eps, momentum, out_dtype, defer,
                           any(ctx.needs_input_grad))
        ctx.save_for_backward(x, *saved)
        ctx.conf = (relu, training, link)
        ctx.mask_in = FUSE and getattr(x, "_acfe_relu_out", False)
        # x is the residual output of a _ConvAddFn whose wgrad can form this
        # BN's backward apply (acfe_conv2d_wgrad_bnbwd with `add`)
        # (the producing node opted in: conv_add(..., single_consumer=True))
        ctx.fold = getattr(x, "_acfe_fold_consumer", None) if FUSE_BN_BWD else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *saved = ctx.saved_tensors
        relu, training, link = ctx.conf
        add = pool = sub = None
        if link is not None:
            add, pool, sub = link.take(), link.take_pool(), link.take_sub()
            if add is None and pool is None and sub is None and not link.declined:
                raise RuntimeError("ResidualLink: the shortcut gradient was not delivered before this BN's backward")
        if ctx.fold is not None and pool is None and sub is None and (link is None or not link.declined):
            # x's only autograd consumer is this BN (a shortcut's gradient came
            # through the link): dx is returned unwritten, its apply pending for
            # the producing conv's backward (_ConvAddFn), which forms it inside
            # its weight gradient or, failing that, runs the apply pass
            dx, dgamma, dbeta = _bn_bwd_pending(x, dy, saved, relu, training, add, ctx.mask_in, ctx.gb)
            ctx.fold.pending = True
        else:
            dx, dgamma, dbeta = _bn_bwd(x, dy, saved, relu, training, add=add, mask_in=ctx.mask_in, pool=pool,
                                        params=ctx.gb, sub=sub)
        return dx, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None


def _bn_bwd_pending(x, dy, saved, relu, training, add, mask_in, params):
    """_bn_bwd up to its apply pass: the reduce (or the slab the producing
    dgrad formed) and the coefficients run now; dx comes back UNWRITTEN with
    the apply's arguments attached (_acfe_bwd_pending), for _take_pending."""
    scale, shift, mean, invstd = saved
    C = x.shape[-1]
    rows = x.numel() // C
    dev = x.device
    nrows = lib.acfe_reduce_blocks(rows)
    prow = nrows
    part = None
    lazy = _tagged(dy, "_acfe_bnpart")
    if lazy is not None and lazy[2] == (x.data_ptr(), tuple(x.shape), bool(relu)):
        part, prow = lazy[0], lazy[1]
    dy = dy.contiguous()
    if part is None:
        part = _empty((nrows * 2 * C,), F64, dev)
        call("acfe_bn_bwd_reduce", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), rows, C, ptr(scale),
             ptr(shift), ptr(mean), ptr(invstd), int(relu), ptr(part), stream())
    coef, dgamma, dbeta = _bn_bwd_coef(part, prow, C, rows, saved, training, params, dev)
    if add is not None:
        add = add.contiguous()
        assert add.dtype == x.dtype and add.shape == x.shape
    dx = _empty(x.shape, x.dtype, dev)
    flags = int(relu) | (2 if mask_in else 0)
    dx._acfe_bwd_pending = ((dy, x, scale, shift, flags, coef, add), dx._version)
    return dx, dgamma, dbeta


def _take_pending(g):
    """The pending BN backward apply of gradient g (None when g is written).
    g must be the very tensor _bn_bwd_pending returned, untouched: an autograd
    accumulation into it would have read unwritten memory."""
    p = getattr(g, "_acfe_bwd_pending", None)
    if p is None:
        return None
    g._acfe_bwd_pending = None
    args, ver = p
    if g._version != ver:
        raise RuntimeError("pending BatchNormalization gradient was modified before its apply ran")
    return args


def _apply_pending(g, args):
    """Write the pending gradient g with the apply pass (acfe_bn_bwd_apply_ex),
    its channel sums attached as _bn_bwd does."""
    dy, x, scale, shift, flags, coef, add = args
    C = x.shape[-1]
    rows = x.numel() // C
    want_sum = FUSE and _sums_ok(g) and _sums_ok(dy) and _sums_ok(x) and (add is None or _sums_ok(add))
    sums = _empty((lib.acfe_reduce_blocks(rows), 2, C), F64, x.device) if want_sum else None
    call("acfe_bn_bwd_apply_ex", ptr(dy), dtype_code(dy.dtype), ptr(x), dtype_code(x.dtype), rows, C, ptr(scale),
         ptr(shift), flags, ptr(coef), ptr(add), 0.0, 0, ptr(g), dtype_code(x.dtype), ptr(sums), stream())
    if want_sum:
        _attach_sum(g, sums, rows)
    if flags & 2:
        _tag(g, "_acfe_relu_masked", True)


def batch_norm(x, gamma, beta, mmean, mvar, training, relu=False, stats=None, eps=1e-3, momentum=0.99, link=None,
               defer=False):
    """defer: return the output pending (see _bn_fwd) -- only for a consumer
    that takes it through bn_prologue_ok's path or materialize()s it."""
    return _BNFn.apply(x, gamma, beta, stats, mmean, mvar, bool(training), bool(relu), float(eps),
                       float(momentum), x.dtype, link, bool(defer))


class _ConvDropBNFn(torch.autograd.Function):
    """BatchNormalization(+ReLU) of Dropout(Conv2D(x)) as one node: the dropout
    and the BN statistics run in the conv epilogue (acfe_conv2d_fwd_dropout),
    the dropout backward inside acfe_bn_bwd_apply_dropout."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, mmean, mvar, conf):
        ctx.bias = b
        ctx.gb = (gamma, beta)
        stride, pt, pl, P, Q, rate, seed, training, relu, eps, momentum, defer = conf
        drop = (rate, seed) if training and rate > 0.0 else None
        ctx.bn = bn_src(x)
        keep = None
        if keep_bits_ok(x, w, stride, pt, pl, P, Q, drop, training) and any(ctx.needs_input_grad):
            # the dropout keep bits for the BN-fold weight gradient (1/16 of u)
            keep = _empty((x.shape[0], P, Q, w.shape[0] // 8), torch.uint8, x.device)
        ctx.keep = keep
        u, stats = _conv_fwd(x, w, b, stride, pt, pl, P, Q, training, drop, keep)
        y, saved = _bn_fwd(u, gamma, beta, stats if training else None, mmean, mvar, training, relu, eps, momentum,
                           u.dtype, defer, any(ctx.needs_input_grad))
        ctx.save_for_backward(x, w, u, *saved)
        ctx.conf = conf
        ctx.has_b = b is not None
        ctx.drop = drop
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, u, *saved = ctx.saved_tensors
        stride, pt, pl, P, Q, rate, seed, training, relu, eps, momentum, _ = ctx.conf
        if _bnbwd_fold_ok(x, w, u, dy, stride, pt, pl, P, Q) and ctx.needs_input_grad[1]:
            return _conv_bn_bwd_fold(ctx, x, w, u, dy, saved, relu, training)
        g, dgamma, dbeta = _bn_bwd(u, dy, saved, relu, training, drop=ctx.drop, params=ctx.gb)
        dx, dw, db = _conv_bwd(x, w, g, stride, pt, pl, P, Q, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               ctx.has_b and ctx.needs_input_grad[2], bias=ctx.bias, bn=ctx.bn)
        return dx, dw, db, dgamma, dbeta, None, None, None


def _bnbwd_fold_ok(x, w, u, dy, stride, pt, pl, P, Q) -> bool:
    """acfe_conv2d_wgrad_bnbwd covers the node: bf16 3x3 stride-1 "same", the
    halo wgrad shapes (acfe_conv2d_wgrad_bnbwd_rows), 16-B aligned operands."""
    if not FUSE_BN_BWD or x.dtype != torch.bfloat16 or u.dtype != x.dtype or dy.dtype != x.dtype:
        return False
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    if (R, S, stride, pt, pl, P, Q) != (3, 3, 1, 1, 1, H, W) or not (x.is_contiguous() and u.is_contiguous()):
        return False
    if u.data_ptr() % 16 or x.data_ptr() % 16 or (dy.is_contiguous() and dy.data_ptr() % 16):
        return False
    return lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K) > 0


def _wgrad_bnbwd(x, w, g, pend, need_db, bias, rate=0.0, seed=0, keep=None):
    """acfe_conv2d_wgrad_bnbwd: dW (and the bias gradient from its channel
    sums) of conv(x, w) whose output gradient g it forms and writes from the
    BN backward apply `pend` = (dy, x_bn, scale, shift, flags, coef, add);
    keep: the forward's dropout keep bits (acfe_conv2d_wgrad_bnbwd_keep)."""
    N, H, W, C = x.shape
    K = w.shape[0]
    dev = x.device
    s = stream()
    dy, u, scale, shift, flags, coef, add = pend
    tgt = direct_grad(w)
    dwt = tgt if tgt is not None else _empty(w.shape, F32, dev)
    ws = _empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), F32, dev)
    srows = lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K)
    sums = _empty((srows, 2, K), F64, dev)
    with _Timed(w, "wgrad"):
        if keep is not None and add is None and rate > 0.0:
            call("acfe_conv2d_wgrad_bnbwd_keep", ptr(x), N, H, W, C, ptr(dy), ptr(u), K, ptr(scale), ptr(shift),
                 int(flags), ptr(coef), float(rate), int(seed), ptr(keep), ptr(g), ptr(dwt),
                 1.0 if tgt is not None else 0.0, ptr(ws), ptr(sums), s)
        else:
            call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(dy), ptr(u), K, ptr(scale), ptr(shift),
                 int(flags), ptr(coef), ptr(add), float(rate), int(seed), ptr(g), ptr(dwt),
                 1.0 if tgt is not None else 0.0, ptr(ws), ptr(sums), s)
    if flags & 2:
        _tag(g, "_acfe_relu_masked", True)
    # g's channel sums: the bias gradient here and of any other conv receiving
    # g (a conv shortcut's, through autograd: channel_sum)
    _attach_sum(g, sums, g.numel() // K, srows)
    dw = dwt
    if tgt is not None:
        dw = None
        grads_ready(w)
    db = None
    if need_db:
        tb = direct_grad(bias)
        out = tb if tb is not None else _empty((K,), F32, dev)
        call("acfe_channel_sum_finalize", ptr(sums), srows, K, 1.0 if tb is not None else 0.0, ptr(out), s)
        db = out
        if tb is not None:
            db = None
            grads_ready(bias)
    return dw, db


def _conv_bn_bwd_fold(ctx, x, w, u, dy, saved, relu, training):
    """Backward of BN(Dropout(Conv2D(x))) with the BN backward apply inside the
    conv's weight gradient (acfe_conv2d_wgrad_bnbwd): the wgrad stages the BN
    output gradient dy and the BN input u, forms the conv output gradient g
    (written for the dgrad, its channel sums = the bias gradient) -- the apply
    pass over the tensor is gone.  Same values as _bn_bwd -> _conv_bwd."""
    N, H, W, C = x.shape
    K = w.shape[0]
    dev = x.device
    s = stream()
    scale, shift, mean, invstd = saved
    rows = u.numel() // K
    dy = dy.contiguous()
    part = None
    prow = nrows = lib.acfe_reduce_blocks(rows)
    lazy = _tagged(dy, "_acfe_bnpart")
    if lazy is not None and lazy[2] == (u.data_ptr(), tuple(u.shape), bool(relu)):
        part, prow = lazy[0], lazy[1]
    if part is None:
        part = _empty((nrows * 2 * K,), F64, dev)
        call("acfe_bn_bwd_reduce", ptr(dy), dtype_code(dy.dtype), ptr(u), dtype_code(u.dtype), rows, K, ptr(scale),
             ptr(shift), ptr(mean), ptr(invstd), int(relu), ptr(part), s)
    coef, dgamma, dbeta = _bn_bwd_coef(part, prow, K, rows, saved, training, ctx.gb, dev)
    g = _empty(u.shape, u.dtype, dev)  # the conv output gradient
    rate, seed = ctx.drop if ctx.drop is not None else (0.0, 0)
    dw, db = _wgrad_bnbwd(x, w, g, (dy, u, scale, shift, int(relu), coef, None),
                          ctx.has_b and ctx.needs_input_grad[2], ctx.bias, rate, seed, getattr(ctx, "keep", None))
    dx = None
    if ctx.needs_input_grad[0]:
        dx, _, _ = _conv_bwd(x, w, g, 1, 1, 1, H, W, True, False, False, bias=ctx.bias, bn=ctx.bn)
    return dx, dw, db, dgamma, dbeta, None, None, None


def conv_dropout_bn(x, w, b, gamma, beta, mmean, mvar, training, rate=0.0, seed=None, relu=True, stride=1,
                    padding="same", eps=1e-3, momentum=0.99, defer=False):
    """BN(Dropout(Conv2D(x))) (+ReLU), Keras semantics of each layer; defer:
    the BN output is returned pending (batch_norm)."""
    if not FUSE:
        u, _ = conv2d(x, w, b, stride, padding)
        u = dropout(u, rate, training, seed)
        return batch_norm(u, gamma, beta, mmean, mvar, training, relu=relu, eps=eps, momentum=momentum)
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    if padding == "same":
        P, pt = same_padding(H, R, stride)
        Q, pl = same_padding(W, S, stride)
    else:
        P, Q, pt, pl = valid_out(H, R, stride), valid_out(W, S, stride), 0, 0
    if training and rate > 0.0 and seed is None:
        seed = next_seed()
    conf = (stride, pt, pl, P, Q, float(rate), int(seed or 0), bool(training), bool(relu), float(eps),
            float(momentum), bool(defer))
    return _ConvDropBNFn.apply(x, w, b, gamma, beta, mmean, mvar, conf)


# ------------------------------------------------------------------ 1x1 conv + BN, conv output recomputed
def _c1bn_ok(x, w, stride) -> bool:
    K, R, S, C = w.shape
    return (FUSE and x.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous() and x.data_ptr() % 16 == 0
            and R == 1 and S == 1 and stride == 1 and w.is_contiguous() and bool(lib.acfe_c1bn_supported(C, K)))


class _C1BNFn(torch.autograd.Function):
    """BatchNormalization(+ReLU) of a 1x1 Conv2D with 16 input channels as one
    node (csrc/c1bn.hip): the conv output is never stored; its statistics come
    from the 16x16 Gram matrix of x, the backward's sums from g^T x.  A pending
    BN output x (the block's bn2a0) is never written: every pass reads the BN
    input and applies the BN (+ReLU) itself (acfe_c1bn_*_bn)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, mmean, mvar, conf):
        ctx.bias = b
        ctx.gb = (gamma, beta)
        training, relu, eps, momentum = conf
        N, H, W, C = x.shape
        K = w.shape[0]
        M = N * H * W
        dev, s = x.device, stream()
        pend = _pending(x)
        if pend is not None and not (PRO_C1 and pend[0].is_contiguous() and pend[0].data_ptr() % 16 == 0
                                     and pend[0].shape == x.shape):
            materialize(x)
            pend = None
        # (x stays pending: a later reader would materialize it)
        xr, xsc, xsh, xrelu = pend if pend is not None else (x, None, None, False)
        scale, shift, mean, invstd = (_empty((K,), F32, dev) for _ in range(4))
        ws = _empty((lib.acfe_c1bn_workspace(M, C, K),), F32, dev)
        gram = _empty((272,), F32, dev)
        part = _empty((1, 2, K), F64, dev)
        if pend is not None:
            call("acfe_c1bn_stats_bn", ptr(xr), M, C, ptr(w), K, ptr(b), ptr(part), ptr(gram), ptr(ws), ptr(xsc),
                 ptr(xsh), int(xrelu), s)
        else:
            call("acfe_c1bn_stats", ptr(x), M, C, ptr(w), K, ptr(b), ptr(part), ptr(gram), ptr(ws), s)
        if training:
            call("acfe_bn_finalize", ptr(part), 1, K, K, float(M), ptr(gamma), ptr(beta), eps, momentum,
                 ptr(mmean), ptr(mvar), 1, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), s)
        else:
            call("acfe_bn_finalize", None, 0, K, K, 0.0, ptr(gamma), ptr(beta), eps, momentum, ptr(mmean),
                 ptr(mvar), 0, ptr(scale), ptr(shift), ptr(mean), ptr(invstd), s)
        y = _empty((N, H, W, K), x.dtype, dev)
        if pend is not None:
            call("acfe_c1bn_apply_bn", ptr(xr), M, C, ptr(w), K, ptr(b), ptr(scale), ptr(shift), int(relu), ptr(y),
                 ptr(xsc), ptr(xsh), int(xrelu), s)
            ctx.save_for_backward(xr, w, b, scale, shift, mean, invstd, gram, xsc, xsh)
        else:
            call("acfe_c1bn_apply", ptr(x), M, C, ptr(w), K, ptr(b), ptr(scale), ptr(shift), int(relu), ptr(y), s)
            ctx.save_for_backward(x, w, b, scale, shift, mean, invstd, gram, None, None)
        ctx.conf = conf
        ctx.xrelu = bool(xrelu)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, scale, shift, mean, invstd, gram, xsc, xsh = ctx.saved_tensors
        training, relu, eps, momentum = ctx.conf
        N, H, W, C = x.shape
        K = w.shape[0]
        M = N * H * W
        dev = x.device
        dy = dy.contiguous()
        dx = _empty(x.shape, x.dtype, dev)
        dw = _empty(w.shape, F32, dev)
        db = _empty((K,), F32, dev) if b is not None else None
        dgamma, dbeta = _empty((K,), F32, dev), _empty((K,), F32, dev)
        ws = _empty((lib.acfe_c1bn_workspace(M, C, K),), F32, dev)
        # eval mode: statistics are constants -> count -> inf removes the mean terms
        args = (ptr(dy), ptr(x), M, C, ptr(w), K, ptr(b), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), int(relu),
                float(M) if training else 1e300, ptr(gram), ptr(dx), ptr(dw), ptr(db), ptr(dgamma), ptr(dbeta),
                ptr(ws))
        if xsc is not None:  # x is the BN input of the prologue; dx is the gradient for its output
            call("acfe_c1bn_bwd_bn", *args, ptr(xsc), ptr(xsh), int(ctx.xrelu), stream())
        else:
            call("acfe_c1bn_bwd", *args, stream())
        return dx, dw, db, dgamma, dbeta, None, None, None


def conv_bn(x, w, b, gamma, beta, mmean, mvar, training, relu=True, stride=1, padding="same", eps=1e-3,
            momentum=0.99, defer=False):
    """BatchNormalization(Conv2D(x)) (+ReLU), Keras semantics of each layer.  A
    bf16 1x1 conv with 16 input channels runs as the recomputing node _C1BNFn;
    anything else as the two layers (conv epilogue statistics -> BN; defer:
    the BN output is returned pending, batch_norm)."""
    if _c1bn_ok(x, w, stride):
        return _C1BNFn.apply(x, w, b, gamma, beta, mmean, mvar,
                             (bool(training), bool(relu), float(eps), float(momentum)))
    u, st = conv2d(x, w, b, stride, padding, want_stats=bool(training))
    return batch_norm(u, gamma, beta, mmean, mvar, training, relu=relu, stats=st if training else None, eps=eps,
                      momentum=momentum, defer=defer)


# ------------------------------------------------------------------ elementwise / pooling
class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, relu, want_stats, link):
        z = torch.empty_like(a)
        stats = _no_stats(a.device)
        C = a.shape[-1]
        if want_stats:
            rows = a.numel() // C
            stats = _empty((lib.acfe_reduce_blocks(rows), 2, C), F64, a.device)
            call("acfe_add_stats", ptr(a), ptr(b), rows, C, int(relu), ptr(z), dtype_code(a.dtype), ptr(stats),
                 stream())
        else:
            call("acfe_add", ptr(a), ptr(b), a.numel(), int(relu), ptr(z), dtype_code(a.dtype), stream())
        ctx.relu, ctx.link = relu, link
        if relu:
            ctx.save_for_backward(z)
            z._acfe_relu_out = True  # a BatchNormalization reading z folds in the ReLU backward
        ctx.mark_non_differentiable(stats)
        return z, stats

    @staticmethod
    def backward(ctx, g, _gs):
        g = g.contiguous()
        if ctx.relu and not _tagged(g, "_acfe_relu_masked"):
            (z,) = ctx.saved_tensors
            d = torch.empty_like(g)
            C = g.shape[-1]
            if FUSE and g.dim() > 1 and _sums_ok(g) and _sums_ok(z) and _sums_ok(d):
                rows = g.numel() // C
                part = _empty((lib.acfe_reduce_blocks(rows), 2, C), F64, g.device)
                call("acfe_relu_bwd_sum", ptr(g), ptr(z), rows, C, ptr(d), dtype_code(g.dtype), ptr(part), stream())
                _attach_sum(d, part, rows)
            else:
                call("acfe_relu_bwd", ptr(g), ptr(z), g.numel(), ptr(d), dtype_code(g.dtype), stream())
            g = d
        if ctx.link is not None:  # the shortcut input's gradient is added by the linked BN backward
            ctx.link.grad = g
            return g, None, None, None, None
        return g, g, None, None, None


def add(a, b, relu=False, want_stats=False, link=None):
    """z = a + b (+ReLU); with want_stats returns (z, BN statistics slab of z).
    `link`: ResidualLink whose BN consumer of `b` adds b's gradient itself."""
    z, st = _AddFn.apply(a.contiguous(), b.contiguous(), bool(relu), bool(want_stats), link)
    return (z, st) if want_stats else z


def _conv_add_ok(x, w, sc, stride, padding) -> bool:
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    return (FUSE and x.dtype == torch.bfloat16 and stride == 1 and padding == "same" and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and sc.dtype == x.dtype and tuple(sc.shape) == (N, H, W, K)
            and sc.is_contiguous() and sc.data_ptr() % 16 == 0
            and (R, S) == (3, 3) and bool(lib.acfe_conv2d_fwd_add_supported(N, H, W, C, K, dtype_code(x.dtype))))


class _ConvAddFn(torch.autograd.Function):
    """(ReLU)(Conv2D 3x3(x) + shortcut) as one node: the residual Add, its ReLU
    and the next BN's statistics run in the conv epilogue (acfe_conv2d_fwd_add);
    the conv output itself is never stored."""

    @staticmethod
    def forward(ctx, x, w, b, sc, relu, want_stats, link, single):
        ctx.bias = b
        ctx.bn = bn_src(x)
        N, H, W, C = x.shape
        K, R, S, _ = w.shape
        _, pt = same_padding(H, R, 1)
        _, pl = same_padding(W, S, 1)
        wp = pack_weights(w, x.dtype, False)
        sc = sc.contiguous()
        z = _empty((N, H, W, K), x.dtype, x.device)
        stats = _no_stats(x.device)
        if want_stats:
            stats = _empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), F64, x.device)
        pro = _pending(x) is not None and bn_prologue_ok(x.shape, x.dtype, w)
        if not pro:
            materialize(x)
        with _Timed(w, "fwd"):
            if pro:  # x is a pending BN output: convolve it through the prologue, which also writes it
                xr, scale, shift, brelu = _prologue_args(x)
                call("acfe_conv2d_fwd_add_bn", ptr(xr), N, H, W, C, ptr(wp), K, pt, pl, ptr(b), ptr(sc), int(relu),
                     ptr(z), ptr(stats) if want_stats else None, ptr(scale), ptr(shift), int(brelu), ptr(x),
                     dtype_code(x.dtype), stream())
            else:
                call("acfe_conv2d_fwd_add", ptr(x), N, H, W, C, ptr(wp), K, pt, pl, ptr(b), ptr(sc), int(relu),
                     ptr(z), ptr(stats) if want_stats else None, dtype_code(x.dtype), stream())
        ctx.save_for_backward(x, w, z if relu else None)
        ctx.conf = (pt, pl, relu, b is not None, link)
        if relu:
            z._acfe_relu_out = True  # a BatchNormalization reading z folds in the ReLU backward
        ctx.fold = None
        if FUSE_BN_BWD and single:
            # the caller guarantees z's only autograd consumer is one BN: its
            # backward apply may be left pending for this node (_FoldToken)
            ctx.fold = z._acfe_fold_consumer = _FoldToken()
        ctx.mark_non_differentiable(stats)
        return z, stats

    @staticmethod
    def backward(ctx, g, _gs):
        x, w, z = ctx.saved_tensors
        pt, pl, relu, has_b, link = ctx.conf
        N, H, W, C = x.shape
        K = w.shape[0]
        pend = _take_pending(g)
        if pend is None and ctx.fold is not None and ctx.fold.pending:
            # the BN left its dx unwritten for this node, but the gradient that
            # arrived is another tensor: z had a second autograd consumer and
            # autograd summed unwritten memory into it
            raise RuntimeError("conv_add(single_consumer=True): the output fed more than one autograd consumer; "
                               "its BatchNormalization gradient was left pending")
        if pend is not None:
            if (ctx.needs_input_grad[1] and _bnbwd_fold_ok(x, w, pend[1], g, 1, pt, pl, H, W)
                    and pend[0].data_ptr() % 16 == 0 and (pend[6] is None or pend[6].data_ptr() % 16 == 0)):
                # the BN backward apply inside this conv's wgrad, writing g
                dw, db = _wgrad_bnbwd(x, w, g, pend, has_b and ctx.needs_input_grad[2], ctx.bias)
                dx = None
                if ctx.needs_input_grad[0]:
                    dx, _, _ = _conv_bwd(x, w, g, 1, pt, pl, H, W, True, False, False, bias=ctx.bias, bn=ctx.bn)
                if link is not None:
                    link.grad = g
                    return dx, dw, db, None, None, None, None, None
                return dx, dw, db, g, None, None, None, None
            _apply_pending(g, pend)
        g = g.contiguous()
        if relu and not _tagged(g, "_acfe_relu_masked"):
            d = torch.empty_like(g)
            if _sums_ok(g) and _sums_ok(z) and _sums_ok(d):
                rows = g.numel() // K
                part = _empty((lib.acfe_reduce_blocks(rows), 2, K), F64, g.device)
                call("acfe_relu_bwd_sum", ptr(g), ptr(z), rows, K, ptr(d), dtype_code(g.dtype), ptr(part), stream())
                _attach_sum(d, part, rows)
            else:
                call("acfe_relu_bwd", ptr(g), ptr(z), g.numel(), ptr(d), dtype_code(g.dtype), stream())
            g = d
        dx, dw, db = _conv_bwd(x, w, g, 1, pt, pl, H, W, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                               has_b and ctx.needs_input_grad[2], bias=ctx.bias, bn=ctx.bn)
        if link is not None:  # the shortcut input's gradient is added by the linked BN backward
            link.grad = g
            return dx, dw, db, None, None, None, None, None
        return dx, dw, db, g, None, None, None, None


class _FoldToken:
    """Shared by a _ConvAddFn node and the BN reading its output: `pending` is
    set when the BN's backward left its dx unwritten for the node."""
    __slots__ = ("pending",)

    def __init__(self):
        self.pending = False


def conv_add(x, w, b, sc, relu=False, want_stats=False, link=None, stride=1, padding="same", single_consumer=False):
    """(ReLU)(Conv2D(x) + sc) -> (z, BN statistics slab of z or empty): one node
    when the conv epilogue covers the shape, else conv2d then add.
    single_consumer: the caller guarantees z's only autograd consumer is one
    batch_norm (the WRN blocks: the next bn2a, the shortcut's gradient through
    its ResidualLink), so that BN's backward apply may be folded into this
    node's weight gradient.  A second consumer then raises in the backward."""
    if _conv_add_ok(x, w, sc, stride, padding):
        return _ConvAddFn.apply(x, w, b, sc, bool(relu), bool(want_stats), link, bool(single_consumer))
    y, _ = conv2d(x, w, b, stride, padding)
    if want_stats:
        return add(y, sc, relu=relu, want_stats=True, link=link)
    return add(y, sc, relu=relu, link=link), _no_stats(x.device)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rate, seed):
        y = torch.empty_like(x)
        call("acfe_dropout", ptr(x), x.numel(), rate, seed, ptr(y), dtype_code(x.dtype), stream())
        ctx.conf = (rate, seed)
        return y

    @staticmethod
    def backward(ctx, g):
        rate, seed = ctx.conf
        g = g.contiguous()
        d = torch.empty_like(g)
        call("acfe_dropout", ptr(g), g.numel(), rate, seed, ptr(d), dtype_code(g.dtype), stream())
        return d, None, None


_seed_counter = itertools.count(1)
_seed_rank = 0


def set_seed_rank(rank: int):
    """Data-parallel replicas draw their own dropout masks (per-replica
    tf.random under MirroredStrategy): the rank enters the seed base."""
    global _seed_rank
    _seed_rank = int(rank) & 0xFF


def next_seed() -> int:
    return (0x5EED << 32) + (_seed_rank << 24) + next(_seed_counter)


def dropout(x, rate, training, seed=None):
    if not training or rate == 0.0:
        return x
    if seed is None:
        seed = next_seed()
    return _DropoutFn.apply(x, float(rate), int(seed))


def _pool_fused_ok(x, kh, kw):
    C = x.shape[-1]
    return ((kh, kw) in ((1, 2), (2, 2), (3, 3)) and C % 8 == 0 and 256 % (C // 8) == 0 and C <= 2048
            and x.data_ptr() % 16 == 0)


def _maxpool_fwd(x, kh, kw, drop, want_stats):
    """acfe_maxpool2d_fused -> (y, argmax bytes, stats slab or empty)."""
    N, H, W, C = x.shape
    P, Q = H // kh, W // kw
    y = _empty((N, P, Q, C), x.dtype, x.device)
    amax = _empty((N, P, Q, C), torch.uint8, x.device)
    stats = _no_stats(x.device)
    if want_stats:
        stats = _empty((lib.acfe_reduce_blocks(N * P * Q), 2, C), F64, x.device)
    rate, seed = drop if drop is not None else (0.0, 0)
    call("acfe_maxpool2d_fused", ptr(x), N, H, W, C, kh, kw, ptr(y), ptr(amax), float(rate), int(seed),
         ptr(stats) if want_stats else None, dtype_code(x.dtype), stream())
    return y, amax, stats


def _maxpool_bwd(amax, g, shape, kh, kw, drop):
    N, H, W, C = shape
    g = g.contiguous()
    dx = _empty(shape, g.dtype, g.device)
    rate, seed = drop if drop is not None else (0.0, 0)
    call("acfe_maxpool2d_bwd_argmax", ptr(amax), ptr(g), N, H, W, C, kh, kw, float(rate), int(seed), ptr(dx),
         dtype_code(g.dtype), stream())
    return dx


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, want_stats):
        ctx.k, ctx.shape = (kh, kw), x.shape
        if (FUSE or want_stats) and _pool_fused_ok(x, kh, kw):
            y, amax, stats = _maxpool_fwd(x, kh, kw, None, want_stats)
            ctx.save_for_backward(amax)
            ctx.fused = True
        else:
            if want_stats:
                raise ValueError("max_pool statistics need C % 8 == 0 and a (1,2)/(2,2)/(3,3) window")
            N, H, W, C = x.shape
            y = _empty((N, H // kh, W // kw, C), x.dtype, x.device)
            call("acfe_maxpool2d", ptr(x), N, H, W, C, kh, kw, ptr(y), dtype_code(x.dtype), stream())
            ctx.save_for_backward(x)
            ctx.fused = False
            stats = _no_stats(x.device)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, g, _gs):
        kh, kw = ctx.k
        if ctx.fused:
            (amax,) = ctx.saved_tensors
            return _maxpool_bwd(amax, g, ctx.shape, kh, kw, None), None, None, None
        (x,) = ctx.saved_tensors
        N, H, W, C = x.shape
        g = g.contiguous()
        dx = torch.empty_like(x)
        call("acfe_maxpool2d_bwd", ptr(x), ptr(g), N, H, W, C, kh, kw, ptr(dx), dtype_code(x.dtype), stream())
        return dx, None, None, None


class _BNPoolFn(torch.autograd.Function):
    """MaxPool2D((kh, kw))(BatchNormalization(x)) (+ReLU) as one node: the
    normalised tensor is formed at load time inside the pooling kernel
    (acfe_bn_maxpool2d_fused) and never stored; the backward expands the pooled
    gradient from the argmax bytes and runs the BN backward on x."""

    @staticmethod
    def forward(ctx, x, gamma, beta, mmean, mvar, stats, conf):
        ctx.gb = (gamma, beta)
        kh, kw, training, relu, eps, momentum, want_stats = conf
        _, saved = _bn_fwd(x, gamma, beta, stats if training else None, mmean, mvar, training, relu, eps, momentum,
                           None)
        N, H, W, C = x.shape
        P, Q = H // kh, W // kw
        y = _empty((N, P, Q, C), x.dtype, x.device)
        amax = _empty((N, P, Q, C), torch.uint8, x.device)
        pst = _no_stats(x.device)
        if want_stats:
            pst = _empty((lib.acfe_reduce_blocks(N * P * Q), 2, C), F64, x.device)
        call("acfe_bn_maxpool2d_fused", ptr(x), N, H, W, C, ptr(saved[0]), ptr(saved[1]), int(relu), kh, kw, ptr(y),
             ptr(amax), ptr(pst) if want_stats else None, dtype_code(x.dtype), stream())
        ctx.save_for_backward(x, amax, *saved)
        ctx.conf = conf
        ctx.mark_non_differentiable(pst)
        return y, pst

    @staticmethod
    def backward(ctx, g, _gs):
        x, amax, *saved = ctx.saved_tensors
        kh, kw, training, relu, eps, momentum, want_stats = ctx.conf
        if FUSE_BN_REDUCE and _sums_ok(x):
            # the pool backward also forms the BN backward's reduce slab (it
            # reads x at the pixels it expands to): no separate reduce pass
            N, H, W, C = x.shape
            g = g.contiguous()
            gu = _empty(x.shape, g.dtype, g.device)
            part = _empty((lib.acfe_reduce_blocks(N * H * W) * 2 * C,), F64, x.device)
            scale, shift, mean, invstd = saved
            call("acfe_maxpool2d_bwd_argmax_bn", ptr(amax), ptr(g), N, H, W, C, kh, kw, ptr(gu), dtype_code(g.dtype),
                 ptr(x), ptr(scale), ptr(shift), ptr(mean), ptr(invstd), int(relu), ptr(part), stream())
            dx, dgamma, dbeta = _bn_bwd(x, gu, saved, relu, training, params=ctx.gb, part=part)
        else:
            gu = _maxpool_bwd(amax, g, x.shape, kh, kw, None)
            dx, dgamma, dbeta = _bn_bwd(x, gu, saved, relu, training, params=ctx.gb)
        return dx, dgamma, dbeta, None, None, None, None


def bn_max_pool(x, gamma, beta, mmean, mvar, training, kh, kw, relu=False, stats=None, eps=1e-3, momentum=0.99,
                want_stats=False):
    """MaxPool2D((kh, kw))(BatchNormalization(x)) (+ReLU) -> (y, stats slab of y
    or None).  wr_resnet_bird.py:29-30 (stem BN -> MaxPool2D((1, 2)))."""
    if not FUSE or not _pool_fused_ok(x, kh, kw):
        y = batch_norm(x, gamma, beta, mmean, mvar, training, relu=relu, stats=stats, eps=eps, momentum=momentum)
        if want_stats:
            return max_pool(y, kh, kw, want_stats=True)
        return max_pool(y, kh, kw), None
    conf = (kh, kw, bool(training), bool(relu), float(eps), float(momentum), bool(want_stats))
    y, st = _BNPoolFn.apply(x, gamma, beta, mmean, mvar, stats, conf)
    return y, (st if want_stats else None)


def max_pool(x, kh, kw, want_stats=False):
    y, st = _MaxPoolFn.apply(x, kh, kw, bool(want_stats))
    return (y, st) if want_stats else y


class _PoolDropBNFn(torch.autograd.Function):
    """BatchNormalization(+ReLU) of Dropout(MaxPool2D(x)) as one node
    (acfe_maxpool2d_fused writes the pooled+dropped values, their argmax
    bytes and BN statistics in one pass; backward from the argmax bytes)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, mmean, mvar, conf):
        ctx.gb = (gamma, beta)
        kh, kw, rate, seed, training, relu, eps, momentum = conf
        drop = (rate, seed) if training and rate > 0.0 else None
        u, amax, stats = _maxpool_fwd(x, kh, kw, drop, training)
        y, saved = _bn_fwd(u, gamma, beta, stats if training else None, mmean, mvar, training, relu, eps, momentum,
                           u.dtype, False, any(ctx.needs_input_grad))
        ctx.save_for_backward(u, amax, *saved)
        ctx.conf, ctx.drop, ctx.shape = conf, drop, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        u, amax, *saved = ctx.saved_tensors
        kh, kw, rate, seed, training, relu, eps, momentum = ctx.conf
        gu, dgamma, dbeta = _bn_bwd(u, dy, saved, relu, training, params=ctx.gb)
        dx = _maxpool_bwd(amax, gu, ctx.shape, kh, kw, ctx.drop)
        return dx, dgamma, dbeta, None, None, None


def maxpool_dropout_bn(x, kh, kw, gamma, beta, mmean, mvar, training, rate=0.0, seed=None, relu=True, eps=1e-3,
                       momentum=0.99):
    """BN(Dropout(MaxPool2D((kh, kw))(x))) (+ReLU)."""
    if not FUSE or not _pool_fused_ok(x, kh, kw):
        y = max_pool(x, kh, kw)
        y = dropout(y, rate, training, seed)
        return batch_norm(y, gamma, beta, mmean, mvar, training, relu=relu, eps=eps, momentum=momentum)
    if training and rate > 0.0 and seed is None:
        seed = next_seed()
    conf = (kh, kw, float(rate), int(seed or 0), bool(training), bool(relu), float(eps), float(momentum))
    return _PoolDropBNFn.apply(x, gamma, beta, mmean, mvar, conf)


def _conv_pool_ok(x, w, stride, padding, kh, kw) -> bool:
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    return (FUSE and x.dtype == torch.bfloat16 and stride == 1 and padding == "same" and (kh, kw) == (2, 2)
            and x.is_contiguous() and x.data_ptr() % 16 == 0
            and bool(lib.acfe_conv2d_pool_supported(N, H, W, C, K, R, S, dtype_code(x.dtype)))
            and bool(lib.acfe_conv2d_pool_supported(N, H, W, K, C, R, S, dtype_code(x.dtype))))


class _ConvPoolBNFn(torch.autograd.Function):
    """BatchNormalization(+ReLU) of Dropout(MaxPool2D(2, 2)(Conv2D 3x3(x))) as one
    node: pooling, dropout and the BN statistics run in the conv epilogue
    (acfe_conv2d_fwd_pool stores only the pooled tensor and its argmax bytes);
    the backward expands the pooled gradient inside the dgrad / wgrad input
    staging (acfe_conv2d_{dgrad,wgrad}_unpool)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, mmean, mvar, conf):
        ctx.bias = b
        ctx.gb = (gamma, beta)
        pt, pl, rate, seed, training, relu, eps, momentum, defer = conf
        pro = PRO_POOL and _pending(x) is not None and bn_prologue_ok(x.shape, x.dtype, w)
        if not pro:
            materialize(x)
        N, H, W, C = x.shape
        K = w.shape[0]
        dev = x.device
        drop = (rate, seed) if training and rate > 0.0 else None
        wp = pack_weights(w, x.dtype, False)
        u = _empty((N, H // 2, W // 2, K), x.dtype, dev)
        amax = _empty((N, H // 2, W // 2, K), torch.uint8, dev)
        stats = _empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), F64, dev) if training else None
        r_, s_ = drop if drop is not None else (0.0, 0)
        with _Timed(w, "fwd"):
            if pro:  # x is a pending BN output: the conv applies it while staging and writes it
                xr, scale, shift, brelu = _prologue_args(x)
                call("acfe_conv2d_fwd_pool_bn", ptr(xr), N, H, W, C, ptr(wp), K, pt, pl, ptr(b), ptr(u), ptr(amax),
                     float(r_), int(s_), ptr(stats), ptr(scale), ptr(shift), int(brelu), ptr(x), dtype_code(x.dtype),
                     stream())
            else:
                call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, pt, pl, ptr(b), ptr(u), ptr(amax),
                     float(r_), int(s_), ptr(stats), dtype_code(x.dtype), stream())
        y, saved = _bn_fwd(u, gamma, beta, stats, mmean, mvar, training, relu, eps, momentum, u.dtype, defer,
                           any(ctx.needs_input_grad))
        ctx.save_for_backward(x, w, u, amax, *saved)
        ctx.conf, ctx.drop, ctx.has_b = conf, drop, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, u, amax, *saved = ctx.saved_tensors
        pt, pl, rate, seed, training, relu, eps, momentum, _ = ctx.conf
        N, H, W, C = x.shape
        K = w.shape[0]
        dev, s = x.device, stream()
        g, dgamma, dbeta = _bn_bwd(u, dy, saved, relu, training, drop=ctx.drop, params=ctx.gb)
        if not UNPOOL:  # materialise the pool backward, then the plain dgrad / wgrad
            dfull = _maxpool_bwd(amax, g, (N, H, W, K), 2, 2, None)
            dx, dw, db = _conv_bwd(x, w, dfull, 1, pt, pl, H, W, ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                   ctx.has_b and ctx.needs_input_grad[2], bias=ctx.bias)
            return dx, dw, db, dgamma, dbeta, None, None, None
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wf = pack_weights(w, x.dtype, True)
            dx = _empty(x.shape, x.dtype, dev)
            with _Timed(w, "dgrad"):
                call("acfe_conv2d_dgrad_unpool", ptr(g), ptr(amax), N, H, W, K, ptr(wf), C, pt, pl, ptr(dx),
                     dtype_code(x.dtype), s)
        if ctx.needs_input_grad[1]:
            tgt = direct_grad(w)
            dw = tgt if tgt is not None else _empty(w.shape, F32, dev)
            ws = _empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), F32, dev)
            with _Timed(w, "wgrad"):
                call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(g), ptr(amax), K, pt, pl, ptr(dw),
                     1.0 if tgt is not None else 0.0, dtype_code(x.dtype), ptr(ws), s)
            if tgt is not None:
                dw = None
                grads_ready(w)
        if ctx.has_b and ctx.needs_input_grad[2]:
            tb = direct_grad(ctx.bias)  # the pool backward scatters: sum of the pooled gradient
            db = channel_sum(g, K, into=tb)
            if tb is not None:
                db = None
                grads_ready(ctx.bias)
        return dx, dw, db, dgamma, dbeta, None, None, None


def conv_maxpool_dropout_bn(x, w, b, stride, padding, kh, kw, gamma, beta, mmean, mvar, training, rate=0.0,
                            seed=None, relu=True, eps=1e-3, momentum=0.99, defer=False):
    """BN(Dropout(MaxPool2D((kh, kw))(Conv2D(x)))) (+ReLU): one node with the
    pooling in the conv epilogue when the kernel covers the shape, else the
    conv followed by maxpool_dropout_bn."""
    if not _conv_pool_ok(x, w, stride, padding, kh, kw):
        y, _ = conv2d(x, w, b, stride, padding)
        return maxpool_dropout_bn(y, kh, kw, gamma, beta, mmean, mvar, training, rate, seed, relu, eps, momentum)
    if training and rate > 0.0 and seed is None:
        seed = next_seed()
    K, R, S, _ = w.shape
    _, pt = same_padding(x.shape[1], R, 1)
    _, pl = same_padding(x.shape[2], S, 1)
    conf = (pt, pl, float(rate), int(seed or 0), bool(training), bool(relu), float(eps), float(momentum),
            bool(defer))
    return _ConvPoolBNFn.apply(x, w, b, gamma, beta, mmean, mvar, conf)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, link):
        N, H, W, C = x.shape
        y = _empty((N, -(-H // k), -(-W // k), C), x.dtype, x.device)
        call("acfe_avgpool2d", ptr(x), N, H, W, C, k, ptr(y), dtype_code(x.dtype), stream())
        ctx.shape, ctx.k, ctx.link = x.shape, k, link
        return y

    @staticmethod
    def backward(ctx, g):
        N, H, W, C = ctx.shape
        g = g.contiguous()
        if ctx.link is not None:  # the linked BN reading x adds the spread-out gradient itself
            ctx.link.pool = (g, ctx.k)
            return None, None, None
        dx = _empty(ctx.shape, g.dtype, g.device)
        call("acfe_avgpool2d_bwd", ptr(g), N, H, W, C, ctx.k, ptr(dx), dtype_code(g.dtype), stream())
        return dx, None, None


def avg_pool_same(x, k, link=None):
    """AveragePooling2D(k, strides=k, "same"); with a ResidualLink the backward
    hands the pooled gradient to the BN that reads x (acfe_bn_bwd_apply_pool)."""
    ok = link is not None and x.dim() == 4 and x.shape[-1] % 8 == 0 and x.data_ptr() % 16 == 0
    if link is not None and not ok:
        link.declined = True  # autograd delivers this gradient instead (ResidualLink.declined)
    return _AvgPoolFn.apply(x, k, link if ok else None)


class _AxisPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, outer, L, inner, sharp, mode):
        y = _empty((outer, inner), F32, x.device)
        call("acfe_axis_pool", ptr(x), dtype_code(x.dtype), outer, L, inner, sharp, mode, ptr(y), stream())
        ctx.save_for_backward(x)
        ctx.conf = (outer, L, inner, sharp, mode)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        outer, L, inner, sharp, mode = ctx.conf
        g = g.contiguous().to(F32)
        dx = torch.empty_like(x)
        call("acfe_axis_pool_bwd", ptr(x), dtype_code(x.dtype), ptr(g), outer, L, inner, sharp, mode, ptr(dx),
             stream())
        return dx, None, None, None, None, None


def logmeanexp(x: torch.Tensor, axis: int, sharpness: float = 5.0) -> torch.Tensor:
    """wr_resnet_bird.logmeanexp (wr_resnet_bird.py:83-87), keepdims=False, fp32 out."""
    shp = list(x.shape)
    outer = 1
    for d in shp[:axis]:
        outer *= d
    inner = 1
    for d in shp[axis + 1:]:
        inner *= d
    y = _AxisPoolFn.apply(x.contiguous(), outer, shp[axis], inner, float(sharpness), 0)
    return y.view(shp[:axis] + shp[axis + 1:])


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """GlobalAveragePooling2D on NHWC -> [N, C] fp32."""
    N, H, W, C = x.shape
    return _AxisPoolFn.apply(x.contiguous(), N, H * W, C, 1.0, 1)


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        B, I = x.shape
        O = w.shape[1]
        z = _empty((B, O), F32, x.device)
        call("acfe_dense_fwd", ptr(x), ptr(w), ptr(b), B, I, O, ptr(z), stream())
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        x, w = ctx.saved_tensors
        B, I = x.shape
        O = w.shape[1]
        dz = dz.contiguous()
        dx = _empty((B, I), F32, x.device) if ctx.needs_input_grad[0] else None
        dw = _empty((I, O), F32, x.device)
        db = _empty((O,), F32, x.device) if ctx.has_b else None
        call("acfe_dense_bwd", ptr(x), ptr(w), ptr(dz), B, I, O, ptr(dx), ptr(dw), ptr(db), stream())
        return dx, dw, db


def dense(x, w, b=None):
    """Dense logits (the sigmoid is applied by sigmoid()/the loss)."""
    return _DenseFn.apply(x.contiguous().to(F32), w, b)


def sigmoid(z: torch.Tensor) -> torch.Tensor:
    p = torch.empty_like(z)
    call("acfe_sigmoid", ptr(z), z.numel(), ptr(p), stream())
    return p


LOSS_MODES = {"bce": 0, "binary": 0, "cce": 1, "categorical": 1}


def loss_and_grad(logits: torch.Tensor, target: torch.Tensor, mode: str = "cce", grad_scale: float | None = None):
    """Keras loss (audiomodel.loss, :1206-1223) on sigmoid(logits): returns
    (loss[1] fp32 device tensor, dL/dlogits).  grad_scale defaults to 1/B
    (the batch mean)."""
    B, L = logits.shape
    loss = _empty((1,), F32, logits.device)
    dz = torch.empty_like(logits)
    ws = _empty((B,), F32, logits.device)
    gs = 1.0 / B if grad_scale is None else grad_scale
    call("acfe_loss", ptr(logits.contiguous()), ptr(target.contiguous().to(F32)), B, L, LOSS_MODES[mode], gs, ptr(loss),
         ptr(dz), ptr(ws), stream())
    return loss, dz


def cast(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if x.dtype == dtype:
        return x
    y = _empty(x.shape, dtype, x.device)
    call("acfe_cast", ptr(x.contiguous()), dtype_code(x.dtype), x.numel(), ptr(y), dtype_code(dtype), stream())
    return y


class _CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return cast(x.contiguous(), dtype)

    @staticmethod
    def backward(ctx, g):
        return cast(g.contiguous(), ctx.src), None


def cast_grad(x, dtype):
    return x if x.dtype == dtype else _CastFn.apply(x, dtype)
