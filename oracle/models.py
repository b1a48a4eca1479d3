"""PyTorch-CPU restatement of the reference model graphs (ORACLE, test-only).

resnet/wr_resnet.py:5-90 and resnet/wr_resnet_bird.py:7-179 written with
torch.nn.functional on NCHW tensors and the Keras semantics of the layers:
  Conv2D "same": out = ceil(n/s), pad_total = max((out-1)s + k - n, 0),
                 pad_before = pad_total // 2 (TF), "valid": no padding;
  BatchNormalization: batch mean / biased variance in training, eps 1e-3,
                 moving = moving*0.99 + batch*0.01;
  MaxPool2D valid; AveragePooling2D "same" (in-bounds average);
  logmeanexp(x, axis, sharpness) = (logsumexp(s x, axis) - log n) / s;
  Dense(sigmoid): returned here as logits.
The input is the reference's 3-channel image (the mel repeated 3x,
tfdataset.py:2053), so the product's channel folding is checked too.
Parameters come from a dict keyed like the product modules' state_dict.

`storage` selects the numerics model: None = plain float math (fp32/fp64 per
the tensors), "bf16" = the mixed-precision storage points of the training
config (tf.keras.mixed_precision "mixed_bfloat16": conv operands and outputs,
BN outputs, pooled / added activations stored in bf16, arithmetic in fp32+).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _pads(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def _q(t, storage):
    return t.to(torch.bfloat16).to(t.dtype) if storage == "bf16" else t


def conv(x, w_krsc, b, stride=1, padding="same", storage=None):
    w = _q(w_krsc, storage).permute(0, 3, 1, 2)  # KRSC -> OIHW
    if padding == "same":
        pt, pb = _pads(x.shape[2], w.shape[2], stride)
        pl, pr = _pads(x.shape[3], w.shape[3], stride)
        x = F.pad(x, (pl, pr, pt, pb))
    return _q(F.conv2d(x, w, b, stride), storage)


def bn(x, p, name, training, relu=False, eps=1e-3, momentum=0.99, state=None, storage=None):
    g, b = p[name + ".gamma"], p[name + ".beta"]
    if training:
        mean = x.mean((0, 2, 3))
        var = x.var((0, 2, 3), unbiased=False)
        if state is not None:
            state[name + ".moving_mean"] = state[name + ".moving_mean"] * momentum + mean.detach() * (1 - momentum)
            state[name + ".moving_variance"] = state[name + ".moving_variance"] * momentum + var.detach() * (1 - momentum)
    else:
        mean, var = state[name + ".moving_mean"], state[name + ".moving_variance"]
    y = (x - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps) * g[None, :, None, None] \
        + b[None, :, None, None]
    return _q(F.relu(y) if relu else y, storage)


def avgpool_same(x, k):
    H, W = x.shape[2:]
    pt, pb = _pads(H, k, k)
    pl, pr = _pads(W, k, k)
    ones = torch.ones((1, 1, H, W), dtype=x.dtype)
    s = F.avg_pool2d(F.pad(x, (pl, pr, pt, pb)), k, k, divisor_override=1)
    c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), k, k, divisor_override=1)
    return s / c


def logmeanexp(x, axis, sharpness=5.0):
    """tfp.math.reduce_logmeanexp(x*s, axis)/s  (wr_resnet_bird.py:83-87)."""
    return (torch.logsumexp(x * sharpness, dim=axis) - math.log(x.shape[axis])) / sharpness


def bird_block(X, p, pre, stride, relu_out, training=True, state=None, storage=None):
    """wr_resnet_bird.basic_block (:103-179) on NCHW X; `pre` = "blocks.{i}."."""
    S = storage
    sc = X
    Y = X
    if stride > 1:
        Y = bn(Y, p, pre + "bn2a0", training, relu=True, state=state, storage=S)
        Y = conv(Y, p[pre + "conv2a0.weight"], p[pre + "conv2a0.bias"], storage=S)
    Y = bn(Y, p, pre + "bn2a", training, relu=True, state=state, storage=S)
    Y = conv(Y, p[pre + "conv21.weight"], p[pre + "conv21.bias"], storage=S)
    if stride > 1:
        Y = F.max_pool2d(Y, stride, stride)
    Y = bn(Y, p, pre + "bn2b", training, relu=True, state=state, storage=S)
    Y = conv(Y, p[pre + "conv2b.weight"], p[pre + "conv2b.bias"], storage=S)
    if pre + "shortcut.weight" in p:
        sc = conv(_q(avgpool_same(sc, stride), S), p[pre + "shortcut.weight"], p[pre + "shortcut.bias"], storage=S)
    X = Y + sc
    if relu_out:
        X = F.relu(X)
    return _q(X, S)


def wr_resnet_bird(x_nchw, p, training=True, state=None, depth=22, k=4, storage=None, head_maps=False):
    """wr_resnet_bird.WRResNet forward (:7-80) -> logits.  p: name -> tensor.
    head_maps: return conv2d_head_3's output [N, classes, h, w] instead (before
    the logmeanexp poolings, :69-74)."""
    n = int((depth - 4) / 6)
    S = storage
    X = conv(x_nchw, p["conv1_1.weight"], p["conv1_1.bias"], storage=S)
    X = bn(X, p, "bn_stem", training, state=state, storage=S)
    X = F.max_pool2d(X, (1, 2), (1, 2))
    bi = 0
    for stage in range(1, 4):
        for d in range(n):
            X = bird_block(X, p, f"blocks.{bi}.", 2 if d == 0 else 1, stage + d > 1, training, state, S)
            bi += 1
    X = bn(X, p, "final_bn", training, relu=True, state=state, storage=S)
    X = conv(X, p["head_conv1.weight"], p["head_conv1.bias"], storage=S)
    X = bn(X, p, "head_bn1", training, state=state, storage=S)
    X = conv(X, p["head_conv2.weight"], p["head_conv2.bias"], storage=S)
    X = bn(X, p, "head_bn2", training, state=state, storage=S)
    X = conv(X, p["head_conv3.weight"], p["head_conv3.bias"], storage=S)
    if head_maps:
        return X
    X = X.permute(0, 2, 3, 1)  # NHWC for the Keras axis numbering of logmeanexp
    X = logmeanexp(X, axis=1)   # [N, W, classes]
    X = logmeanexp(X, axis=2)   # [N, W]
    return X @ p["prediction.kernel"] + p["prediction.bias"]


def wrn_block(X, p, pre, stride, training=True, state=None, storage=None):
    """wr_resnet.basic_block (:46-90) on NCHW X; `pre` = "blocks.{i}."."""
    S = storage
    Y = bn(X, p, pre + "bn2a", training, relu=True, state=state, storage=S)
    Y = conv(Y, p[pre + "conv2a.weight"], p[pre + "conv2a.bias"], stride, storage=S)
    Y = bn(Y, p, pre + "bn2b", training, relu=True, state=state, storage=S)
    Y = conv(Y, p[pre + "conv2b.weight"], p[pre + "conv2b.bias"], storage=S)
    sc = X
    if pre + "shortcut.weight" in p:
        sc = conv(X, p[pre + "shortcut.weight"], p[pre + "shortcut.bias"], stride, "valid", storage=S)
    return _q(F.relu(Y + sc), S)


def wr_resnet(x_nchw, p, training=True, state=None, depth=22, k=4, storage=None):
    """wr_resnet.WRResNet forward (:5-33) -> logits."""
    n = int((depth - 4) / 6)
    S = storage
    X = conv(x_nchw, p["conv1_1.weight"], p["conv1_1.bias"], storage=S)
    bi = 0
    for stage in range(1, 4):
        for d in range(n):
            X = wrn_block(X, p, f"blocks.{bi}.", stage if d == 0 else 1, training, state, S)
            bi += 1
    X = bn(X, p, "final_bn", training, relu=True, state=state, storage=S)
    X = X.mean((2, 3))
    return X @ p["prediction.kernel"] + p["prediction.bias"]


def keras_loss(logits, y, mode="cce"):
    """audiomodel.loss (:1206-1223) on sigmoid outputs: BCE (from the logits,
    as Keras does for a sigmoid output) or CCE (renormalised, clipped)."""
    if mode == "bce":
        l = torch.clamp(logits, min=0) - logits * y + torch.log1p(torch.exp(-logits.abs()))
        return l.mean()
    p = torch.sigmoid(logits)
    q = p / p.sum(-1, keepdim=True)
    q = torch.clamp(q, 1e-7, 1 - 1e-7)
    return (-(y * torch.log(q)).sum(-1)).mean()


def keras_adam(params, grads, m, v, t, lr=0.01, b1=0.9, b2=0.999, eps=1e-7):
    """tf.keras.optimizers.Adam update (Keras 3 formulation)."""
    alpha = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    for i in range(len(params)):
        m[i] = m[i] + (grads[i] - m[i]) * (1 - b1)
        v[i] = v[i] + (grads[i] ** 2 - v[i]) * (1 - b2)
        params[i] = params[i] - alpha * m[i] / (torch.sqrt(v[i]) + eps)
    return params, m, v
