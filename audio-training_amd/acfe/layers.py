"""Keras-layer equivalents (tf.keras.layers.Conv2D / BatchNormalization / Dense)
as torch Modules running on the acfe kernels.  Parameter names and layouts:
conv kernel KRSC fp32 (Keras stores RSCK; see to_keras/from_keras), Dense
kernel [in][out] as in Keras, BN gamma/beta/moving_mean/moving_variance."""
from __future__ import annotations

import math
import zlib

import torch
from torch import nn

from . import ops
from .arena import ParamArena  # noqa: F401  (HIP-free, re-exported)


def _pair(k):
    return (k, k) if isinstance(k, int) else tuple(k)


def glorot_uniform(shape, fan_in, fan_out, seed):
    """tf.keras.initializers.GlorotUniform: U(-l, l), l = sqrt(6/(fan_in+fan_out))."""
    g = torch.Generator().manual_seed(int(seed))
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1).mul_(lim).to(torch.float32)


def _seed(name, base=0):
    return (zlib.crc32(name.encode()) + base) & 0x7FFFFFFF


class Conv2D(nn.Module):
    """tf.keras.layers.Conv2D(filters, kernel_size, strides, padding, use_bias=True)."""

    def __init__(self, cin, filters, kernel_size, strides=1, padding="same", use_bias=True, name="conv2d", seed=0):
        super().__init__()
        kh, kw = _pair(kernel_size)
        self.strides, self.padding, self.name = int(strides), padding, name
        self.weight = nn.Parameter(glorot_uniform((filters, kh, kw, cin), kh * kw * cin, kh * kw * filters,
                                                  _seed(name, seed)))
        self.bias = nn.Parameter(torch.zeros(filters)) if use_bias else None

    def forward(self, x, want_stats=False, link=None):
        y, st = ops.conv2d(x, self.weight, self.bias, self.strides, self.padding, want_stats, link=link)
        return (y, st) if want_stats else y


class StemConv2D(Conv2D):
    """First Conv2D of both WRN variants.  Its input has `cin` identical channels
    (tfdataset.py:2053 repeats the mel image 3x); the kernel keeps the Keras
    parameter shape [16, R, S, cin] but runs on the single folded channel."""

    def __init__(self, cin, filters, kernel_size, name="conv1_1", seed=0, out_dtype=torch.bfloat16):
        super().__init__(cin, filters, kernel_size, 1, "same", True, name, seed)
        if filters != 16:
            raise ValueError("the stem kernel is specialised to 16 output channels")
        self.out_dtype = out_dtype

    def forward(self, x, want_stats=False):
        y, st = ops.stem_conv(x, self.weight, self.bias, self.out_dtype, want_stats)
        return (y, st) if want_stats else y


class BatchNormalization(nn.Module):
    """tf.keras.layers.BatchNormalization(axis=3): eps 1e-3, momentum 0.99."""

    def __init__(self, channels, name="batch_normalization", eps=1e-3, momentum=0.99):
        super().__init__()
        self.name, self.eps, self.momentum = name, eps, momentum
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))

    def forward(self, x, relu=False, stats=None, link=None, defer=False):
        """defer: the output comes back pending for a consuming conv's BN
        prologue (ops.batch_norm)."""
        return ops.batch_norm(x, self.gamma, self.beta, self.moving_mean, self.moving_variance, self.training,
                              relu, stats, self.eps, self.momentum, link, defer)


def conv_dropout_bn(conv: Conv2D, bn: BatchNormalization, x, rate, relu=True, defer=False):
    """bn(Dropout(rate)(conv(x))) (+ReLU) as one fused node (ops.conv_dropout_bn)."""
    return ops.conv_dropout_bn(x, conv.weight, conv.bias, bn.gamma, bn.beta, bn.moving_mean, bn.moving_variance,
                               bn.training, rate, relu=relu, stride=conv.strides, padding=conv.padding,
                               eps=bn.eps, momentum=bn.momentum, defer=defer)


def conv_bn(conv: Conv2D, bn: BatchNormalization, x, relu=True, defer=False):
    """bn(conv(x)) (+ReLU) as one node (ops.conv_bn: the recomputing 1x1 node
    when the conv has 16 input channels)."""
    return ops.conv_bn(x, conv.weight, conv.bias, bn.gamma, bn.beta, bn.moving_mean, bn.moving_variance, bn.training,
                       relu=relu, stride=conv.strides, padding=conv.padding, eps=bn.eps, momentum=bn.momentum,
                       defer=defer)


def maxpool_dropout_bn(x, kh, kw, bn: BatchNormalization, rate, relu=True):
    """bn(Dropout(rate)(MaxPool2D((kh, kw))(x))) (+ReLU) as one fused node."""
    return ops.maxpool_dropout_bn(x, kh, kw, bn.gamma, bn.beta, bn.moving_mean, bn.moving_variance, bn.training,
                                  rate, relu=relu, eps=bn.eps, momentum=bn.momentum)


def conv_maxpool_dropout_bn(conv: Conv2D, x, k, bn: BatchNormalization, rate, relu=True, defer=False):
    """bn(Dropout(rate)(MaxPool2D((k, k))(conv(x)))) (+ReLU) as one fused node
    (the pooling runs in the conv epilogue when the kernel covers the shape)."""
    return ops.conv_maxpool_dropout_bn(x, conv.weight, conv.bias, conv.strides, conv.padding, k, k, bn.gamma, bn.beta,
                                       bn.moving_mean, bn.moving_variance, bn.training, rate, relu=relu, eps=bn.eps,
                                       momentum=bn.momentum, defer=defer)


class Dense(nn.Module):
    """tf.keras.layers.Dense(units) logits; the sigmoid of the reference's
    Dense(activation="sigmoid") is applied by predict()/the loss."""

    def __init__(self, cin, units, name="dense", seed=0):
        super().__init__()
        self.name = name
        self.kernel = nn.Parameter(glorot_uniform((cin, units), cin, units, _seed(name, seed)))
        self.bias = nn.Parameter(torch.zeros(units))

    def forward(self, x):
        return ops.dense(x, self.kernel, self.bias)


class Adam:
    """tf.keras.optimizers.Adam(learning_rate=lr) (audiomodel.py:1226-1240):
    beta_1 0.9, beta_2 0.999, epsilon 1e-7, one fused kernel over the arena."""

    def __init__(self, arena: ParamArena, lr=0.01, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.arena, self.lr, self.b1, self.b2, self.eps = arena, lr, beta_1, beta_2, epsilon
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)
        self.iterations = 0

    def step(self, grad_scale=1.0):
        from ._lib import call
        from ._torch import ptr, stream

        self.iterations += 1
        t = self.iterations
        alpha = self.lr * math.sqrt(1.0 - self.b2 ** t) / (1.0 - self.b1 ** t)
        a = self.arena
        call("acfe_adam_step", ptr(a.flat), ptr(a.grad), ptr(self.m), ptr(self.v), a.numel, float(grad_scale),
             self.b1, self.b2, self.eps, float(alpha), stream())
