"""BirdNET-style wide ResNet (reference: resnet/wr_resnet_bird.py:7-179) on the
acfe kernels.

Reproduced reference behaviour (not "fixed"):
  * FILTERS = [8,16,32,64,128] * k is list repetition, so FILTERS[-1] = 128 (:10-12);
  * `filters=X.shape[1]` uses the current HEIGHT as the channel count of the
    2a0 / 21 convolutions (:128, :139);
  * no ReLU after the stem BatchNormalization (:29-30), none after the Add of
    stage 1 block 0 (:177-178);
  * the second logmeanexp(axis=2) runs on the [B, W, classes] result of the
    first (keepdims=False), i.e. it pools the CLASS axis and the Dense sees the
    W positions (:73-77).
Input: the mel image as ONE channel [N, H(=mels), W(=frames)]; the reference's
3 identical channels are folded into the stem kernel (StemConv2D).
"""
from __future__ import annotations

import torch
from torch import nn

from acfe import ops
from acfe.layers import (BatchNormalization, Conv2D, Dense, StemConv2D, conv_bn, conv_dropout_bn,
                         conv_maxpool_dropout_bn)


class BasicBlock(nn.Module):
    """wr_resnet_bird.basic_block (:103-179)."""

    def __init__(self, cin, height, filters, kernel_size, stage, block, sub_id, stride, dropout=0.1, seed=0):
        super().__init__()
        cb, bb = f"res{stage}{block}_branch", f"bn{stage}{block}_branch"
        self.stride, self.dropout = stride, dropout
        c = cin
        if stride > 1:
            self.bn2a0 = BatchNormalization(c, bb + "2a0")
            self.conv2a0 = Conv2D(c, height, (1, 1), 1, "same", name=cb + "2a0", seed=seed)
            c = height
        self.bn2a = BatchNormalization(c, bb + "2a")
        self.conv21 = Conv2D(c, height, kernel_size, 1, "same", name=cb + "21", seed=seed)
        self.bn2b = BatchNormalization(height, bb + "2b")
        self.conv2b = Conv2D(height, filters, kernel_size, 1, "same", name=cb + "2b", seed=seed)
        self.shortcut = None
        if cin != filters:
            self.shortcut = Conv2D(cin, filters, 1, 1, "same", name=f"conv2d_shortcut_{stage}{block}", seed=seed)
            self.shortcut.keras_auto = True  # unnamed in the reference (:169-174): Keras auto-names it
        self.relu_out = stage + sub_id > 1
        self.out_channels = filters
        self.out_height = height // stride if stride > 1 else height

    def forward(self, x, x_stats=None):
        """x -> (block output, its BN statistics slab in training else None).
        Fused nodes: conv21 + Dropout + bn2b (stride 1) or MaxPool + Dropout +
        bn2b (stride 2) in one pass each; the Add writes the statistics the
        next block's first BN consumes; with an identity shortcut the Add's
        gradient for x is summed inside that BN's backward (ResidualLink)."""
        training = self.training
        # identity shortcut: the Add's gradient for x, conv shortcut: the pooled
        # gradient of its AveragePooling2D, both summed inside the BN reading x
        link = ops.ResidualLink.make()
        # BN -> ReLU -> 3x3 conv: the BN output comes back pending and the conv
        # applies it in its input staging (ops.bn_prologue_ok shapes; other
        # consumers write it with the apply pass first)
        defer = ops.FUSE and ops.PROLOGUE
        y = x
        if self.stride > 1:
            y = self.bn2a0(y, relu=True, stats=x_stats, link=link, defer=defer)
            y = conv_bn(self.conv2a0, self.bn2a, y, relu=True, defer=defer)
            y = conv_maxpool_dropout_bn(self.conv21, y, self.stride, self.bn2b, self.dropout, defer=defer)
        else:
            y = self.bn2a(y, relu=True, stats=x_stats, link=link, defer=defer)
            y = conv_dropout_bn(self.conv21, self.bn2b, y, self.dropout, defer=defer)
        # the shortcut is built after the residual branch (its backward then runs
        # first, delivering the linked gradient before the BN reading x needs it)
        sc = x
        if self.shortcut is not None:
            sc = self.shortcut(ops.avg_pool_same(x, self.stride, link=link))
        add_link = link if self.shortcut is None else None
        want = training and ops.FUSE
        z, st = ops.conv_add(y, self.conv2b.weight, self.conv2b.bias, sc, relu=self.relu_out, want_stats=want,
                             single_consumer=True, link=add_link, stride=self.conv2b.strides,
                             padding=self.conv2b.padding)
        return z, (st if want else None)


class WRResNet(nn.Module):
    """WRResNet(input_shape, classes, depth=22, k=4) of wr_resnet_bird.py:7-80.
    forward(x [N,H,W] one folded channel, compute dtype) -> logits [N, classes]
    (the reference's Dense(sigmoid) output is sigmoid(logits))."""

    def __init__(self, input_shape=(120, 512, 1), classes=6, depth=22, k=4, dtype=torch.bfloat16, dropout=0.1,
                 seed=0):
        super().__init__()
        H, W, cin = input_shape
        self.input_shape, self.classes, self.dtype, self.dropout = tuple(input_shape), classes, dtype, dropout
        filters = [16, 16 * k, 32 * k, 64 * k]
        FILTERS = [8, 16, 32, 64, 128] * k
        FILTERS[0] = 8
        n = int((depth - 4) / 6)
        self.conv1_1 = StemConv2D(cin, filters[0], (5, 5), name="conv1_1", seed=seed, out_dtype=dtype)
        self.bn_stem = BatchNormalization(filters[0], "batch_normalization")
        self.bn_stem.keras_auto = True
        h, w, c = H, W // 2, filters[0]
        blocks = []
        for stage in range(1, len(filters)):
            for d in range(n):
                sub = d
                stride = 2 if d == 0 else 1
                blk = BasicBlock(c, h, filters[stage], (3, 3), stage, f"b{d}", sub, stride, dropout, seed)
                blocks.append(blk)
                c, h = blk.out_channels, blk.out_height
                if stride > 1:
                    w = w // stride
        self.blocks = nn.ModuleList(blocks)
        self.final_bn = BatchNormalization(c, "final_bn")
        self.head_conv1 = Conv2D(c, FILTERS[-1], (4, 10), 1, "same", name="conv2d_head_1", seed=seed)
        self.head_bn1 = BatchNormalization(FILTERS[-1], "batch_normalization_head_1")
        self.head_conv2 = Conv2D(FILTERS[-1], FILTERS[-1] * 2, 1, 1, "same", name="conv2d_head_2", seed=seed)
        self.head_bn2 = BatchNormalization(FILTERS[-1] * 2, "batch_normalization_head_2")
        self.head_conv3 = Conv2D(FILTERS[-1] * 2, classes, 1, 1, "same", name="conv2d_head_3", seed=seed)
        self.prediction = Dense(w, classes, name="prediction", seed=seed)
        self.feature_hw = (h, w)
        # layers the reference leaves unnamed (:47-70): matched by class and
        # creation order when Keras weight files are read (keras_weights.py)
        for m in (self.head_conv1, self.head_bn1, self.head_conv2, self.head_bn2, self.head_conv3):
            m.keras_auto = True

    def forward(self, x):
        y = self.head_maps(x)
        y = ops.logmeanexp(y, axis=1, sharpness=5)  # [N, W, classes]
        y = ops.logmeanexp(y, axis=2, sharpness=5)  # [N, W]   (class axis, as in the reference)
        return self.prediction(y)

    def head_maps(self, x):
        """The per-pixel class maps [N, h, w, classes] of conv2d_head_3
        (wr_resnet_bird.py:69-70), before the two logmeanexp poolings."""
        if x.dim() == 4:
            x = x[..., 0]
        bn, c1 = self.bn_stem, self.conv1_1
        if self.training and ops.stem_bn_pool_ok(x, c1.weight, c1.bias, c1.out_dtype, 1, 2):
            # conv1_1 -> BN -> MaxPool2D((1, 2)) as one node: its backward applies
            # the BN backward inside the stem's dgrad / wgrad staging
            y, st = ops.stem_bn_max_pool(x, c1.weight, c1.bias, c1.out_dtype, bn.gamma, bn.beta, bn.moving_mean,
                                         bn.moving_variance, 1, 2, eps=bn.eps, momentum=bn.momentum, want_stats=True)
        else:
            y, st = c1(x, want_stats=True)
            # BN -> MaxPool2D((1, 2)) as one node: the normalised stem output is never stored
            y, st = ops.bn_max_pool(y, bn.gamma, bn.beta, bn.moving_mean, bn.moving_variance, self.training, 1, 2,
                                    stats=st, eps=bn.eps, momentum=bn.momentum, want_stats=self.training)
        for blk in self.blocks:
            y, st = blk(y, st)
        y = self.final_bn(y, relu=True, stats=st)
        y, st = self.head_conv1(y, want_stats=True)
        y = self.head_bn1(y, stats=st)
        y = ops.dropout(y, self.dropout, self.training)
        y, st = self.head_conv2(y, want_stats=True)
        y = self.head_bn2(y, stats=st)
        y = ops.dropout(y, self.dropout, self.training)
        return self.head_conv3(y)

    def predict(self, x):
        return ops.sigmoid(self.forward(x))


def flops_per_clip(model: WRResNet) -> float:
    """Forward conv FLOPs (2*MACs) per clip for the model's input shape."""
    H, W, cin = model.input_shape
    total = 2.0 * 5 * 5 * cin * 16 * H * W
    h, w = H, W // 2
    for blk in model.blocks:
        def conv(c):
            k, r, s, ci = c.weight.shape
            return 2.0 * k * r * s * ci
        if blk.stride > 1:
            total += conv(blk.conv2a0) * h * w + conv(blk.conv21) * h * w
            h, w = h // blk.stride, w // blk.stride
        else:
            total += conv(blk.conv21) * h * w
        total += conv(blk.conv2b) * h * w
        if blk.shortcut is not None:
            total += conv(blk.shortcut) * h * w
    for c in (model.head_conv1, model.head_conv2, model.head_conv3):
        k, r, s, ci = c.weight.shape
        total += 2.0 * k * r * s * ci * h * w
    return total
