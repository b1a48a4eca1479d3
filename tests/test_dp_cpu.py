"""Data-parallel semantics on CPU with the gloo backend (world_size 2), through
the same HIP-free modules the GPU trainer uses (acfe.dp, acfe.arena,
audiomodel.train_epoch):

* allreduce_mean_: the all-reduced, 1/world-scaled flat gradient of two
  replicas equals the gradient of the concatenated batch (oracle WRN model,
  eval-mode BN: no batch coupling), and the Keras-Adam update applied on both
  replicas keeps them bit-identical;
* GradBuckets over a ParamArena: parameters whose gradient a "kernel" writes
  in place into the arena (the ops.direct_grad path, reported explicitly) and
  parameters autograd accumulates (post-accumulate hooks) together; buckets
  launch in reverse arena order DURING the backward (before the last report),
  the summed arena equals the full-batch gradient, and reports arriving in a
  different order on each rank still give the same collective sequence;
* synced_batches / train_epoch over uneven TFRecord shards (AudioDataset with
  file and record sharding, mix_up pairs): every rank runs the same number of
  steps, each with a collective, and nothing hangs;
* average_buffers: BN moving statistics become the replica mean.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _spawn(fn, world=2, *args):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(fn, args=(world, _free_port(), out, *args), nprocs=world, join=True)
    return dict(out)


# ------------------------------------------------------------ allreduce_mean_
def _wrn_params():
    """Parameters of the WRN model without importing the HIP modules: the
    oracle model keyed like the product state_dict."""
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    from oracle.models import wr_resnet  # noqa: F401

    g = torch.Generator().manual_seed(0)
    p, names = {}, []

    def conv(name, cin, k, r):
        p[name + ".weight"] = torch.randn((k, r, r, cin), generator=g, dtype=torch.float64) * (2.0 / (r * r * cin)) ** 0.5
        p[name + ".bias"] = torch.randn((k,), generator=g, dtype=torch.float64) * 0.05
        names.extend([name + ".weight", name + ".bias"])

    def bn(name, c):
        p[name + ".gamma"] = 1 + 0.1 * torch.randn((c,), generator=g, dtype=torch.float64)
        p[name + ".beta"] = 0.05 * torch.randn((c,), generator=g, dtype=torch.float64)
        p[name + ".moving_mean"] = 0.1 * torch.randn((c,), generator=g, dtype=torch.float64)
        p[name + ".moving_variance"] = 1 + 0.5 * torch.rand((c,), generator=g, dtype=torch.float64)
        names.extend([name + ".gamma", name + ".beta"])

    conv("conv1_1", 3, 16, 3)
    c, bi = 16, 0
    for stage, f in zip(range(1, 4), (64, 128, 256)):
        for d in range(3):
            pre = f"blocks.{bi}."
            bn(pre + "bn2a", c)
            conv(pre + "conv2a", c, f, 3)
            bn(pre + "bn2b", f)
            conv(pre + "conv2b", f, f, 3)
            if c != f:
                conv(pre + "shortcut", c, f, 1)
            c = f
            bi += 1
    bn("final_bn", c)
    p["prediction.kernel"] = torch.randn((c, 4), generator=g, dtype=torch.float64) * 0.1
    p["prediction.bias"] = torch.zeros(4, dtype=torch.float64)
    names.extend(["prediction.kernel", "prediction.bias"])
    return p, names


def _grads(p, names, x, y):
    from oracle import models as om

    prm = {k: (v.clone().requires_grad_(True) if k in names else v.clone()) for k, v in p.items()}
    state = {k: v for k, v in prm.items() if "moving" in k}
    z = om.wr_resnet(x[:, None].repeat(1, 3, 1, 1), prm, False, state)
    om.keras_loss(z, y, "cce").backward()
    return torch.cat([prm[n].grad.reshape(-1) for n in names])


def _data():
    g = torch.Generator().manual_seed(5)
    x = torch.randn((4, 32, 24), generator=g, dtype=torch.float64)
    y = torch.zeros((4, 4), dtype=torch.float64)
    y[torch.arange(4), torch.tensor([0, 3, 1, 2])] = 1
    return x, y


def _w_allreduce(rank, world, port, out):
    _init(rank, world, port)
    from acfe.dp import allreduce_mean_
    from oracle.models import keras_adam

    p, names = _wrn_params()
    x, y = _data()
    half = x.shape[0] // world
    flat = _grads(p, names, x[rank * half:(rank + 1) * half], y[rank * half:(rank + 1) * half])
    flat *= allreduce_mean_(flat)
    params = [p[n].clone() for n in names]
    grads, o = [], 0
    for q in params:
        grads.append(flat[o:o + q.numel()].view_as(q))
        o += q.numel()
    new, _, _ = keras_adam(params, grads, [torch.zeros_like(q) for q in params],
                           [torch.zeros_like(q) for q in params], 1)
    out[rank] = (flat.clone(), torch.cat([q.reshape(-1) for q in new]))
    dist.destroy_process_group()


def test_allreduce_mean_equals_full_batch_gradient():
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    out = _spawn(_w_allreduce)
    p, names = _wrn_params()
    x, y = _data()
    full = _grads(p, names, x, y)
    g0, p0 = out[0]
    g1, p1 = out[1]
    assert torch.equal(g0, g1)
    torch.testing.assert_close(g0, full, rtol=1e-10, atol=1e-12)
    assert torch.equal(p0, p1)


# ------------------------------------------------------------ GradBuckets
class _DirectLinear(torch.autograd.Function):
    """y = x W^T + b whose backward accumulates dW / db straight into the arena
    views (as the wgrad / BN-finalize kernels do, ops.direct_grad) and returns
    None for them, reporting readiness like ops.grads_ready."""

    @staticmethod
    def forward(ctx, x, w, b, report):
        ctx.save_for_backward(x, w)
        ctx.b, ctx.report = b, report
        return x @ w.T + b

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        w.grad.add_(g.T @ x)
        ctx.report(w)
        ctx.b.grad.add_(g.sum(0))
        ctx.report(ctx.b)
        return g @ w, None, None, None


class _Layer(torch.nn.Module):
    def __init__(self, cin, cout, g):
        super().__init__()
        self.w = torch.nn.Parameter(torch.randn((cout, cin), generator=g) * 0.3)
        self.b = torch.nn.Parameter(torch.zeros(cout))


class _Net(torch.nn.Module):
    """Parameters registered layer by layer (forward order), as the models do."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(11)
        dims = [12, 40, 40, 40, 40, 6]
        self.layers = torch.nn.ModuleList(_Layer(dims[i], dims[i + 1], g) for i in range(len(dims) - 1))
        self.report = None

    def forward(self, x):
        for i, l in enumerate(self.layers):
            if i % 2 == 0 and self.report is not None:   # in-place "kernel" path
                x = _DirectLinear.apply(x, l.w, l.b, self.report)
            else:                                         # autograd-accumulated path
                x = x @ l.w.T + l.b
            if i < len(self.layers) - 1:
                x = torch.tanh(x)
        return x


def _net_batch():
    g = torch.Generator().manual_seed(12)
    return torch.randn((8, 12), generator=g), torch.randn((8, 6), generator=g)


def _w_buckets(rank, world, port, out):
    _init(rank, world, port)
    from acfe.arena import ParamArena
    from acfe.dp import GradBuckets

    net = _Net()
    arena = ParamArena(net, "cpu")
    # ~1 KB buckets: several buckets over the 5-layer net
    bk = GradBuckets(arena.grad, arena.params, arena.offsets, bucket_bytes=1024)
    order = []

    def report(p):
        # a parameter may be reported twice (in-place writer + autograd's hook,
        # which fires even when the Function returned None): first report counts
        i = next(i for i, q in enumerate(arena.params) if q is p)
        if i not in order:
            order.append(i)
        bk.ready(p)

    for p in arena.params:
        p.register_post_accumulate_grad_hook(report)
    net.report = report
    x, y = _net_batch()
    half = x.shape[0] // world
    for step in range(2):
        arena.zero_grad()
        bk.begin()
        order.clear()
        loss = ((net(x[rank * half:(rank + 1) * half]) - y[rank * half:(rank + 1) * half]) ** 2).sum() / x.shape[0]
        loss.backward()
        reports_before_finish = bk.reports
        scale = bk.finish()
    out[rank] = dict(grad=arena.grad.clone() * scale * world, launch=list(bk.launch_log), nb=len(bk.buckets),
                     reports=reports_before_finish, nparams=len(arena.params), order=list(order),
                     buckets=list(bk.buckets))
    dist.destroy_process_group()


def test_grad_buckets_overlap_and_order():
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    out = _spawn(_w_buckets)
    net = _Net()
    x, y = _net_batch()
    (((net(x) - y) ** 2).sum() / x.shape[0]).backward()
    full = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    for r in (0, 1):
        o = out[r]
        # the sum of both replicas' half-batch gradients = the full-batch gradient
        torch.testing.assert_close(o["grad"], full, rtol=1e-5, atol=1e-6)
        assert o["nb"] >= 3
        # every bucket launched once, in index order (same collective sequence on all ranks)
        assert [b for b, _ in o["launch"]] == list(range(o["nb"]))
        # overlap: the first buckets went out while later gradients were still pending
        early = sum(1 for _, seen in o["launch"] if seen < o["nparams"])
        assert o["launch"][0][1] < o["nparams"] and early >= o["nb"] - 2, o["launch"]
        assert o["reports"] == o["nparams"]
        # bucket 0 holds the LAST parameters of the arena (produced first by backward)
        lo, hi = o["buckets"][0]
        assert hi == sum(p.numel() for p in net.parameters())
        # backward reported the output layer's parameters before the input layer's
        assert o["order"].index(len(o["order"]) - 1) < o["order"].index(0)
    assert out[0]["launch"] == out[1]["launch"]


def _w_shuffled_reports(rank, world, port, out):
    """Reports in a different order per rank: launches still in bucket order."""
    _init(rank, world, port)
    from acfe.dp import GradBuckets

    n = [5, 300, 7, 900, 64, 1000, 3]
    offs, o = [], 0
    for k in n:
        offs.append((o, k))
        o += k
    grad = torch.arange(o, dtype=torch.float64) * (rank + 1)
    params = [object() for _ in n]
    bk = GradBuckets(grad, params, offs, bucket_bytes=8 * 1000)
    perm = list(range(len(n)))
    if rank == 1:
        perm = perm[::-1]
    else:
        perm = [3, 0, 6, 2, 5, 1, 4]
    for i in perm:
        bk.ready(params[i])
        bk.ready(params[i])  # duplicate reports are ignored
    bk.finish()
    out[rank] = (grad.clone(), [b for b, _ in bk.launch_log])
    dist.destroy_process_group()


def test_grad_buckets_report_order_independent():
    out = _spawn(_w_shuffled_reports)
    total = sum([5, 300, 7, 900, 64, 1000, 3])
    ref = torch.arange(total, dtype=torch.float64) * 3
    for r in (0, 1):
        assert torch.equal(out[r][0], ref)
        assert out[r][1] == list(range(len(out[r][1])))


# ------------------------------------------------------------ uneven shards
def _write_shards(root, counts, labels=("bird", "noise")):
    import numpy as np
    import tfrecord as tfr

    root.mkdir(parents=True, exist_ok=True)
    k = 0
    for i, c in enumerate(counts):
        with tfr.TFRecordWriter(root / f"{i:05d}.tfrecord") as w:
            for _ in range(c):
                raw = np.full(144000, 0.001 * (k % 97), np.float32)
                lab = labels[k % len(labels)]
                w.write(tfr.audio_example(raw, f"r{k}", k, lab, lab))
                k += 1
    return k


def _w_epoch(rank, world, port, out, root, augment, record_level):
    _init(rank, world, port)
    import audiomodel
    import tfdataset
    from acfe import dp

    files, shard = audiomodel.shard_files(tfdataset._files(root), rank, world)
    assert (shard is not None) == record_level
    ds = tfdataset.AudioDataset(files, ["bird", "noise"], batch_size=2, shuffle=True, augment=augment,
                                device="cpu", threads=2, drop_remainder=True, seed=3, record_shard=shard)
    ctrl = dp.control_group()
    calls = []

    def step(x1, y1, x2, y2, lam):
        # stands in for Trainer.step: one collective per step on every rank
        t = torch.ones(1)
        dist.all_reduce(t)
        calls.append(int(t.item()))
        return (x1.mean() + (0 if x2 is None else x2.mean())).reshape(1)

    def mixup(b):
        return torch.full((b,), 0.3)

    res = []
    for epoch in range(2):
        res.append(audiomodel.train_epoch(ds, step, augment, 0, mixup, ctrl))
    n_own = sum(1 for f in files for _ in __import__("tfrecord").read_records(f))
    out[rank] = dict(res=res, calls=calls, own=n_own)
    dist.destroy_process_group()


@pytest.mark.parametrize("augment", [False, True], ids=["plain", "mixup"])
@pytest.mark.parametrize("counts,record_level", [((9, 2, 5), False), ((7,), True)], ids=["files", "records"])
def test_uneven_shards_same_step_count(tmp_path, augment, counts, record_level):
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    _write_shards(tmp_path / "train", counts)
    out = _spawn(_w_epoch, 2, str(tmp_path / "train"), augment, record_level)
    s0, s1 = [r[2] for r in out[0]["res"]], [r[2] for r in out[1]["res"]]
    assert s0 == s1 and all(s > 0 for s in s0)
    assert out[0]["calls"] == out[1]["calls"] and all(c == 2 for c in out[0]["calls"])
    # the shorter shard bounds the epoch: no rank got more batches than its records allow
    for r in (0, 1):
        assert s0[0] * 2 <= out[r]["own"]
    if not record_level:  # the ranks' shards really are uneven (9+5 vs 2 records)
        assert out[0]["own"] != out[1]["own"]


def _w_buffers(rank, world, port, out):
    _init(rank, world, port)
    from acfe.dp import average_buffers

    m = torch.nn.Module()
    m.register_buffer("moving_mean", torch.full((3,), float(rank)))
    m.register_buffer("moving_variance", torch.full((3,), 1.0 + 2 * rank))
    m.register_buffer("other", torch.full((3,), float(rank)))
    average_buffers(m)
    out[rank] = (m.moving_mean.clone(), m.moving_variance.clone(), m.other.clone())
    dist.destroy_process_group()


def test_average_buffers():
    out = _spawn(_w_buffers)
    for r in (0, 1):
        mm, mv, other = out[r]
        assert torch.equal(mm, torch.full((3,), 0.5))
        assert torch.equal(mv, torch.full((3,), 2.0))
        assert torch.equal(other, torch.full((3,), float(r)))  # not a BN statistic: untouched
