"""Data-parallel plumbing of the training step (HIP-free: torch.distributed only).

The reference trains on one GPU; the MirroredStrategy line it would have used
is commented out (audiomodel.py:498-500).  Here one process drives one GPU,
the batch is sharded across ranks and the gradient exchange is RCCL (backend
"nccl") over xGMI on the GPU, gloo in the CPU tests.

GradBuckets: the flat fp32 gradient arena (layers.ParamArena) is cut at
parameter boundaries into ~4 MB buckets in REVERSE arena order -- backward
produces the head's gradients first -- and each bucket's in-place all-reduce
(sum) is launched, asynchronously, as soon as the last of its parameters
reports its gradient written.  Reports come from the kernels that accumulate
straight into the arena (acfe.ops.grads_ready) and from autograd's
post-accumulate hooks for the rest.  Buckets are launched strictly in index
order, so every rank issues the same collective sequence whatever order its
reports arrive in; finish() launches what is left (parameters that got no
gradient keep their zeros) and makes the current stream wait for all of them.
The 1/world mean is folded into the Adam kernel (grad_scale), not applied here.

synced_batches: every rank must run the same number of steps (each step has
collectives); a per-step MIN all-reduce of a "have a batch" host flag over a
gloo group stops all ranks at the first exhausted shard (uneven TFRecord
shards, mix_up pairs that stop early, more ranks than files) without a
device synchronisation.

average_buffers: Keras keeps BatchNormalization moving statistics SyncOnRead
(MEAN) under MirroredStrategy, so a saved model holds the replica mean; this
averages the moving_* buffers across ranks before evaluation / saving.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

BUCKET_BYTES = 4 << 20  # ~4 MB buckets


def world_size(group=None) -> int:
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def allreduce_mean_(flat: torch.Tensor, group=None) -> float:
    """Sum-all-reduce `flat` in place (one collective); returns the factor
    (1/world) that turns the sum into the mean of the replicas' batch-mean
    gradients (applied inside the Adam kernel)."""
    world = world_size(group)
    if world == 1:
        return 1.0
    dist.all_reduce(flat, group=group)
    return 1.0 / world


class GradBuckets:
    """Bucketed, backward-overlapped all-reduce of a flat gradient arena.

    grad: the flat fp32 gradient buffer; params / offsets: the arena's
    parameters and their (offset, numel) in it, in arena (forward) order."""

    def __init__(self, grad: torch.Tensor, params, offsets, bucket_bytes=BUCKET_BYTES, group=None):
        self.grad, self.group = grad, group
        self.world = world_size(group)
        cap = max(1, bucket_bytes // grad.element_size())
        self.buckets: list[tuple[int, int]] = []   # [lo, hi) ranges of the arena
        self.members: list[int] = []               # parameter count per bucket
        self.index: dict[int, int] = {}            # id(param) -> bucket
        lo = hi = None
        count = 0
        for p, (o, n) in reversed(list(zip(params, offsets))):
            if hi is not None and (hi - o) > cap and count:
                self.buckets.append((lo, hi))
                self.members.append(count)
                hi, count = None, 0
            if hi is None:
                hi = o + n
            lo = o
            count += 1
            self.index[id(p)] = len(self.buckets)
        if hi is not None:
            self.buckets.append((lo, hi))
            self.members.append(count)
        self.launch_log: list[tuple[int, int]] = []  # (bucket, reports seen at launch) of the last step
        self.begin()

    def begin(self):
        self.left = list(self.members)
        self.seen: set[int] = set()
        self.next = 0
        self.works = []
        self.reports = 0
        self.launch_log = []

    def _launch(self, b):
        lo, hi = self.buckets[b]
        self.launch_log.append((b, self.reports))
        if self.world > 1:
            self.works.append(dist.all_reduce(self.grad[lo:hi], group=self.group, async_op=True))

    def ready(self, p):
        """Parameter p's gradient is fully written (its producing kernels are
        enqueued on the current stream)."""
        k = id(p)
        b = self.index.get(k)
        if b is None or k in self.seen:
            return
        self.seen.add(k)
        self.reports += 1
        self.left[b] -= 1
        while self.next < len(self.buckets) and self.left[self.next] == 0:
            self._launch(self.next)
            self.next += 1

    def finish(self) -> float:
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        for w in self.works:
            w.wait()
        self.works = []
        return 1.0 / self.world


def control_group():
    """A gloo (host-side) group for per-step control flags: exchanging them
    over RCCL would make the host wait for the GPU queue every step."""
    if world_size() == 1:
        return None
    if dist.get_backend() == "gloo":
        return dist.group.WORLD
    return dist.new_group(backend="gloo")


def synced_batches(iterable, group=None):
    """Yield items of `iterable` while EVERY rank still has one: a per-step
    MIN all-reduce of a one-element host flag over `group` (a gloo group,
    control_group()); single-process: plain iteration."""
    world = world_size(group)
    it = iter(iterable)
    if world == 1:
        yield from it
        return
    flag = torch.ones(1, dtype=torch.int32)
    while True:
        item = next(it, None)
        flag.fill_(0 if item is None else 1)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) == 0:
            return
        yield item


def average_buffers(module: torch.nn.Module, suffixes=("moving_mean", "moving_variance"), group=None):
    """Mean of the BN moving statistics over ranks, in place (Keras SyncOnRead MEAN)."""
    world = world_size(group)
    if world == 1:
        return
    bufs = [b for n, b in module.named_buffers() if n.endswith(suffixes)]
    if not bufs:
        return
    flat = torch.cat([b.reshape(-1).float() for b in bufs])
    dist.all_reduce(flat, group=group)
    flat /= world
    o = 0
    with torch.no_grad():
        for b in bufs:
            n = b.numel()
            b.copy_(flat[o:o + n].view_as(b))
            o += n


def allreduce_sums(values, device=None, group=None):
    """Sum a few host floats over ranks (sharded evaluation totals)."""
    if world_size(group) == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, group=group)
    return t.tolist()
