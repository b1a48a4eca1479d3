"""One rank of tests/test_dp_gpu.py (not collected by pytest: no test_ prefix).

Started as a fresh child process (never forked or exec'd from a process that
has touched the GPU) with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment.  Every rank runs on cuda:0 with the gloo backend (RCCL refuses two
ranks on one device); the HIP Trainer and its GradBuckets are the production
ones: the bucket all-reduces are launched during the backward from the
kernels' grads_ready reports and the autograd post-accumulate hooks.

Writes {grad, params, loss, launch_log, reports, buckets} to argv[1].<rank>.pt.
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT), str(ROOT / "tests")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dp_case  # noqa: E402


def rccl_single_rank(out_prefix):
    """RCCL (backend "nccl") on this box's one GPU: a one-rank group runs the
    production GradBuckets path with the collective forced on (the bucket
    all-reduces of a real backward, launched from the kernels' reports), so
    the library, its stream handling and the in-place bucket views execute;
    with one rank the sum must leave the gradient unchanged."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from acfe import dp

    tr = dp_case.make_trainer(dev)
    tr.buckets = dp.GradBuckets(tr.arena.grad, tr.arena.params, tr.arena.offsets, dp_case.BUCKET_BYTES)
    tr.buckets.world = 2  # force the all-reduce launches (the group itself has one rank)
    for p in tr.arena.params:
        p.register_post_accumulate_grad_hook(tr._grad_done)
    x1, x2, lam, y = dp_case.batch(dev, 0, 1)
    loss, _ = tr.step(x1, y, x2, lam)
    torch.cuda.synchronize()
    torch.save({"grad": tr.arena.grad.detach().cpu().clone(), "loss": float(loss),
                "launch_log": list(tr.buckets.launch_log), "backend": dist.get_backend()}, f"{out_prefix}.rccl.pt")
    print(f"rccl: {len(tr.buckets.launch_log)} bucket all-reduces over {dist.get_backend()}", flush=True)
    dist.destroy_process_group()


def main(out_prefix):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if os.environ.get("ACFE_DP_TEST") == "rccl1":
        return rccl_single_rank(out_prefix)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from acfe import ops

    ops.set_seed_rank(rank)
    training = os.environ.get("ACFE_DP_BN") == "train"
    tr = dp_case.make_trainer(dev, bucket_bytes=dp_case.BUCKET_BYTES, training=training)
    assert tr.buckets is not None and tr.world == world
    x1, x2, lam, y = dp_case.batch(dev, rank, world)
    print(f"rank {rank}: step 1", flush=True)
    loss, _ = tr.step(x1, y, x2, lam)
    torch.cuda.synchronize()
    # the all-reduced (summed) gradient arena the Adam step just consumed, and
    # the parameters after Adam (grad_scale 1/world)
    res = {"grad": tr.arena.grad.detach().cpu().clone(), "params": tr.arena.flat.detach().cpu().clone(),
           "loss": float(loss), "launch_log": list(tr.buckets.launch_log), "reports": tr.buckets.reports,
           "buckets": list(tr.buckets.buckets)}
    torch.save(res, f"{out_prefix}.{rank}.pt")
    print(f"rank {rank}: done, {len(res['launch_log'])} buckets", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
