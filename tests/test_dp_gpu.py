"""Data-parallel correctness of the real HIP Trainer on the GPU (VERDICT r02
next #2; the reference's MirroredStrategy line, audiomodel.py:498-500).

Two ranks are started as fresh child processes (tests/dp_gpu_worker.py) BEFORE
this process touches the GPU; both run on cuda:0 with the gloo backend (RCCL
refuses two ranks on one device; the collective sequence, the bucket
machinery and the Trainer are the production ones).  Each rank trains one step
on its half of the global batch (dropout 0, per-replica PCEN min/max as
MirroredStrategy would run it; BatchNormalization in eval mode, and once more
in training mode with per-replica batch statistics).  This process then recomputes, on
one GPU without any collective, the arena gradient of each half and checks:

* the all-reduced arena on every rank == g(half 0) + g(half 1) bit for bit
  (a sum of two fp32 values is order-independent, and every kernel of the
  backward reduces in a fixed order);
* the replicas' parameters after Adam (grad_scale 1/world) are bit-identical
  to each other and to a single-process Adam step on that summed gradient;
* every bucket was launched once, in bucket order, the first one before the
  backward's last gradient report (overlap with the backward);
* no bucket is launched before its last contribution: a bucket's gradient
  snapshotted (stream-ordered clone) at launch time equals its final value,
  including the parameters that receive both a kernel report and autograd
  accumulations (stem, Dense, PCEN, the 1x1+BN node).
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

WORKER = Path(__file__).resolve().parent / "dp_gpu_worker.py"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(tmp_path_factory, bn_mode):
    if torch.cuda.device_count() < 1:  # counting devices does not initialise HIP
        pytest.skip("no GPU")
    out = tmp_path_factory.mktemp("dp") / "res"
    world, port = 2, _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), ACFE_DP_BN=bn_mode)
        procs.append(subprocess.Popen([sys.executable, "-u", str(WORKER), str(out)], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(p.wait())
    assert rcs == [0] * world, rcs
    return [torch.load(f"{out}.{r}.pt", weights_only=True) for r in range(world)]


@pytest.fixture(scope="module")
def rank_results(tmp_path_factory):
    return _run_ranks(tmp_path_factory, "eval")


@pytest.fixture(scope="module")
def rank_results_train(tmp_path_factory):
    """The same two ranks with training-mode BatchNormalization: each replica
    normalises with its own half-batch statistics (Keras MirroredStrategy's
    default non-synced BN)."""
    return _run_ranks(tmp_path_factory, "train")


@pytest.fixture(scope="module")
def rccl_result(rank_results, tmp_path_factory):
    """A one-rank RCCL group (this box has one GPU) in a fresh child process,
    started after the gloo pair has exited and before this process touches
    the GPU."""
    out = tmp_path_factory.mktemp("rccl") / "res"
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), ACFE_DP_TEST="rccl1")
    p = subprocess.Popen([sys.executable, "-u", str(WORKER), str(out)], env=env)
    try:
        rc = p.wait(timeout=240)
    except subprocess.TimeoutExpired:
        p.kill()
        rc = p.wait()
    assert rc == 0, rc
    return torch.load(f"{out}.rccl.pt", weights_only=True)


def _half_grads(tr, dev, world):
    """Each rank's half-batch gradient recomputed in this process (in the
    trainer's BN mode: training mode normalises each half with its own
    statistics, as each replica does)."""
    from acfe import ops

    import dp_case

    grads, losses = [], []
    for r in range(world):
        x1, x2, lam, y = dp_case.batch(dev, r, world)
        tr.arena.zero_grad()
        feats = tr.frontend(x1, x2, lam)
        z = tr.model(feats)
        loss, dz = ops.loss_and_grad(z, y, tr.loss_mode)
        z.backward(dz)
        grads.append(tr.arena.grad.detach().clone())
        losses.append(float(loss))
    return grads, losses


def test_rccl_bucket_allreduce_executes(rccl_result, cuda):
    """RCCL ran the bucketed all-reduce of a real HIP backward (one rank: the
    summed gradient equals the local one, which this process recomputes)."""
    import dp_case

    assert rccl_result["backend"] == "nccl"
    assert [b for b, _ in rccl_result["launch_log"]] == list(range(len(rccl_result["launch_log"])))
    assert len(rccl_result["launch_log"]) >= 3
    tr = dp_case.make_trainer(cuda)
    g, _ = _half_grads(tr, cuda, 1)
    assert torch.equal(rccl_result["grad"], g[0].cpu())


@pytest.mark.parametrize("bn_mode", ["eval", "train"])
def test_dp_step_matches_single_process(request, cuda, bn_mode):
    import dp_case

    rank_results = request.getfixturevalue("rank_results" if bn_mode == "eval" else "rank_results_train")
    world = len(rank_results)
    tr = dp_case.make_trainer(cuda, training=bn_mode == "train")
    assert tr.buckets is None  # single process: no collective
    p0 = tr.arena.flat.detach().clone()
    grads, losses = _half_grads(tr, cuda, world)
    gsum = grads[0] + grads[1]
    for r, res in enumerate(rank_results):
        assert abs(res["loss"] - losses[r]) <= 1e-6 * max(1.0, abs(losses[r])), (r, res["loss"], losses[r])
        assert torch.equal(res["grad"], gsum.cpu()), (r, (res["grad"] - gsum.cpu()).abs().max())
    # replicas bit-identical after Adam, and equal to one Adam step on the sum
    assert torch.equal(rank_results[0]["params"], rank_results[1]["params"])
    with torch.no_grad():
        tr.arena.flat.copy_(p0)
        tr.arena.grad.copy_(gsum)
    tr.opt.step(grad_scale=1.0 / world)
    torch.cuda.synchronize()
    assert torch.equal(rank_results[0]["params"], tr.arena.flat.detach().cpu())
    # the gradient of the concatenated batch is the mean of the half-batch ones
    # up to the per-replica PCEN min/max (eval-mode BN couples nothing else)
    assert not torch.equal(rank_results[0]["params"], p0.cpu())


def test_dp_bucket_launch_order(rank_results):
    for res in rank_results:
        nb = len(res["buckets"])
        assert nb >= 3
        assert [b for b, _ in res["launch_log"]] == list(range(nb))
        # the first bucket (the head's gradients) goes out while the backward
        # is still reporting gradients
        assert res["launch_log"][0][1] < res["reports"]
    assert rank_results[0]["launch_log"] == rank_results[1]["launch_log"]


def test_no_bucket_launches_before_its_last_contribution(cuda):
    """Single process, the Trainer's bucket path with a recording subclass:
    each bucket's gradient is cloned on the launch stream when it is launched;
    after the backward every clone must equal the final gradient (a late
    kernel accumulation or autograd add into a launched bucket would differ)."""
    from acfe import dp

    import dp_case

    class Recording(dp.GradBuckets):
        def _launch(self, b):
            lo, hi = self.buckets[b]
            self.snap.append((b, self.grad[lo:hi].detach().clone()))
            super()._launch(b)

    tr = dp_case.make_trainer(cuda)
    rb = Recording(tr.arena.grad, tr.arena.params, tr.arena.offsets, dp_case.BUCKET_BYTES)
    rb.snap = []
    tr.buckets = rb
    for p in tr.arena.params:
        p.register_post_accumulate_grad_hook(tr._grad_done)
    x1, x2, lam, y = dp_case.batch(cuda, 0, 1)
    for _ in range(2):  # the second step runs with the WeightPacker
        rb.snap = []
        tr.step(x1, y, x2, lam)
        torch.cuda.synchronize()
        assert [b for b, _ in rb.snap] == list(range(len(rb.buckets)))
        assert rb.launch_log[0][1] < rb.reports  # overlapped with the backward
        for b, s in rb.snap:
            lo, hi = rb.buckets[b]
            assert torch.equal(s, tr.arena.grad[lo:hi]), b
        # every arena parameter reported exactly once
        assert rb.reports == len(tr.arena.params)
