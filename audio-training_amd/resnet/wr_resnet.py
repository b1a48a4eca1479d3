"""Wide ResNet WRN-22-4 (reference: resnet/wr_resnet.py:5-90) on the acfe kernels.

Pre-activation basic blocks (BN-ReLU-Conv3x3(stride)-Dropout-BN-ReLU-Conv3x3
+ identity or 1x1 strided "valid" shortcut, ReLU after the Add); stage strides
1, 2, 3 (wr_resnet.py:21-23); BN-ReLU-GlobalAveragePooling-Dense(sigmoid) head.
Input: the mel image as ONE channel [N, H, W] (the 3 identical channels of
tfdataset.py:2053 are folded into the stem kernel)."""
from __future__ import annotations

import torch
from torch import nn

from acfe import ops
from acfe.layers import BatchNormalization, Conv2D, Dense, StemConv2D, conv_dropout_bn


class BasicBlock(nn.Module):
    """wr_resnet.basic_block (:46-90)."""

    def __init__(self, cin, filters, stage, block, stride, dropout=0.1, seed=0):
        super().__init__()
        F1, F2 = filters
        cb, bb = f"res{stage}{block}_branch", f"bn{stage}{block}_branch"
        self.stride, self.dropout = stride, dropout
        self.bn2a = BatchNormalization(cin, bb + "2a")
        self.conv2a = Conv2D(cin, F1, (3, 3), stride, "same", name=cb + "2a", seed=seed)
        self.bn2b = BatchNormalization(F1, bb + "2b")
        self.conv2b = Conv2D(F1, F2, (3, 3), 1, "same", name=cb + "2b", seed=seed)
        self.shortcut = None
        if cin != F2:
            # Keras default padding "valid", default (unseeded) GlorotUniform
            self.shortcut = Conv2D(cin, F2, 1, stride, "valid", name=f"conv2d_shortcut_{stage}{block}", seed=seed + 1)
            self.shortcut.keras_auto = True  # unnamed in the reference (:84-86): Keras auto-names it
        self.out_channels = F2

    def forward(self, x, x_stats=None):
        """x -> (block output, its BN statistics slab in training else None);
        conv2a + Dropout + bn2b run as one fused node (ops.conv_dropout_bn),
        conv2b + the residual Add + ReLU (+ the next BN's statistics) as
        another (ops.conv_add: the rows kernel's Add epilogue where it covers
        the shape, else conv2d -> add).  A conv shortcut's gradient reaches x
        through autograd's accumulation; the gradient-tensor tags the fused
        nodes rely on are version-checked (ops._tag)."""
        # the gradient of x from the shortcut (the Add's, or the 1x1 conv
        # shortcut's dX) is summed inside bn2a's backward (ResidualLink), with
        # the ReLU mask of x when x is the previous block's ReLU output
        link = ops.ResidualLink.make()
        # BN outputs come back pending: the 3x3 convs apply them in their input
        # staging where ops.bn_prologue_ok covers the shape
        defer = ops.FUSE and ops.PROLOGUE
        y = self.bn2a(x, relu=True, stats=x_stats, link=link, defer=defer)
        y = conv_dropout_bn(self.conv2a, self.bn2b, y, self.dropout, defer=defer)
        # (created after bn2a: its backward runs first and delivers the link)
        sc = x if self.shortcut is None else self.shortcut(x, link=link)
        want = self.training and ops.FUSE
        z, st = ops.conv_add(y, self.conv2b.weight, self.conv2b.bias, sc, relu=True, want_stats=want,
                             single_consumer=True, link=link if self.shortcut is None else None,
                             stride=self.conv2b.strides, padding=self.conv2b.padding)
        return z, (st if want else None)


class WRResNet(nn.Module):
    """WRResNet(input_shape, classes, depth=22, k=4) of wr_resnet.py:5-33."""

    def __init__(self, input_shape=(128, 512, 1), classes=6, depth=22, k=4, dtype=torch.bfloat16, dropout=0.1,
                 seed=0):
        super().__init__()
        H, W, cin = input_shape
        self.input_shape, self.classes, self.dtype, self.dropout = tuple(input_shape), classes, dtype, dropout
        filters = [16, 16 * k, 32 * k, 64 * k]
        n = int((depth - 4) / 6)
        self.conv1_1 = StemConv2D(cin, filters[0], (3, 3), name="conv1_1", seed=seed, out_dtype=dtype)
        c = filters[0]
        blocks = []
        for stage in range(1, len(filters)):
            f = filters[stage]
            for d in range(n):
                stride = stage if d == 0 else 1
                blk = BasicBlock(c, (f, f), stage + 1, f"b{d}", stride, dropout, seed)
                blocks.append(blk)
                c = blk.out_channels
        self.blocks = nn.ModuleList(blocks)
        self.final_bn = BatchNormalization(c, "final_bn")
        self.prediction = Dense(c, classes, name="prediction", seed=seed)

    def forward(self, x):
        if x.dim() == 4:
            x = x[..., 0]
        y, st = self.conv1_1(x, want_stats=True)
        if not self.training:
            st = None
        for blk in self.blocks:
            y, st = blk(y, st)
        y = self.final_bn(y, relu=True, stats=st)
        y = ops.global_avg_pool(y)
        return self.prediction(y)

    def predict(self, x):
        return ops.sigmoid(self.forward(x))
