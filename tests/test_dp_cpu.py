"""Data-parallel semantics on CPU with the gloo backend (world_size 2):
the all-reduced, 1/world-scaled flat gradient arena of two replicas equals the
gradient of the concatenated batch (no batch coupling: eval-mode BN), and the
Keras-Adam update applied on both replicas keeps them bit-identical.  Uses the
same `allreduce_mean_` the HIP trainer calls, on the oracle model."""
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


def _params():
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    torch.manual_seed(0)
    from resnet.wr_resnet import WRResNet

    m = WRResNet(input_shape=(32, 24, 3), classes=4, dropout=0.0)
    p = {k: v.detach().double().clone() for k, v in m.state_dict().items()}
    names = [n for n, _ in m.named_parameters()]
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


def _worker(rank, world, port, out):
    import sys

    sys.path[:0] = [str(PKG), str(ROOT)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from acfe_dp import allreduce_mean_  # noqa: F401  (module alias set below)

    p, names = _params()
    x, y = _data()
    half = x.shape[0] // world
    flat = _grads(p, names, x[rank * half:(rank + 1) * half], y[rank * half:(rank + 1) * half])
    scale = allreduce_mean_(flat)
    flat *= scale
    # identical Adam step on both replicas
    from oracle.models import keras_adam

    params = [p[n].clone() for n in names]
    grads, o = [], 0
    for q in params:
        grads.append(flat[o:o + q.numel()].view_as(q))
        o += q.numel()
    new, _, _ = keras_adam(params, grads, [torch.zeros_like(q) for q in params],
                           [torch.zeros_like(q) for q in params], 1)
    out[rank] = (flat.clone(), torch.cat([q.reshape(-1) for q in new]))
    dist.destroy_process_group()


def test_allreduce_mean_equals_full_batch_gradient(tmp_path):
    import sys
    import types

    # expose train.allreduce_mean_ without importing the HIP library in the workers
    src = (PKG / "acfe" / "train.py").read_text()
    start = src.index("def allreduce_mean_")
    end = src.index("class Trainer")
    (tmp_path / "acfe_dp.py").write_text("import torch\n\n" + src[start:end])
    sys.path.insert(0, str(tmp_path))
    os.environ["PYTHONPATH"] = os.pathsep.join([str(tmp_path), str(PKG), str(ROOT), os.environ.get("PYTHONPATH", "")])
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    p, names = _params()
    x, y = _data()
    full = _grads(p, names, x, y)
    g0, p0 = out[0]
    g1, p1 = out[1]
    assert torch.equal(g0, g1)
    torch.testing.assert_close(g0, full, rtol=1e-10, atol=1e-12)
    assert torch.equal(p0, p1)
