"""Flat parameter / gradient arena (HIP-free; acfe.layers re-exports it).

All trainable parameters of a module become views of ONE flat fp32 buffer and
their gradients views of one flat gradient buffer, so the data-parallel
all-reduce runs over contiguous buckets of one tensor (acfe.dp.GradBuckets)
and Adam is one kernel launch over the whole model (acfe.layers.Adam).
"""
from __future__ import annotations

import torch
from torch import nn


class ParamArena:
    """All trainable parameters of a module as views of ONE flat fp32 buffer,
    with gradients as views of one flat gradient buffer: the data-parallel
    all-reduce is a single (bucketable) collective and Adam one kernel launch."""

    def __init__(self, module: nn.Module, device):
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        o = 0
        self.offsets = []
        with torch.no_grad():
            for p in self.params:
                n = p.numel()
                self.flat[o:o + n].copy_(p.detach().reshape(-1).to(device))
                p.data = self.flat[o:o + n].view(p.shape)
                p.grad = self.grad[o:o + n].view(p.shape)
                p._acfe_arena = True  # ops.direct_grad: kernels may accumulate into p.grad
                self.offsets.append((o, n))
                o += n

    def zero_grad(self):
        self.grad.zero_()
        for p, (o, n) in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:].data_ptr():
                p.grad = self.grad[o:o + n].view(p.shape)
