#!/usr/bin/env python3
"""Per-parameter gradient error of the HIP model step against the float64
oracle (and the float32 oracle's own error e32), for one test configuration.
usage: python tools/model_grad_report.py [bird|wrn] [f32|bf16] [train|eval]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "audio-training_amd"), str(ROOT), str(ROOT / "tests")]
import torch  # noqa: E402

import test_model_gpu as t  # noqa: E402
from oracle import models as om  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "bird"
    dtype = torch.float32 if (sys.argv[2] if len(sys.argv) > 2 else "f32") == "f32" else torch.bfloat16
    training = (sys.argv[3] if len(sys.argv) > 3 else "eval") == "train"
    cuda = torch.device("cuda", 0)
    H, W, classes, N = 128, 64, 10, 2
    m = t._build(kind, (H, W, 3), classes, dtype, cuda)
    m.train(training)
    x = t._input(N, H, W)
    tgt = torch.zeros(N, classes, dtype=torch.float64)
    tgt[0, 3] = tgt[1, 7] = 1
    fwd = om.wr_resnet_bird if kind == "bird" else om.wr_resnet

    def oracle(dt):
        p = {k: v.detach().to(dt).cpu().clone() for k, v in m.state_dict().items()}
        prm = {k: v.requires_grad_(True) for k, v in p.items() if "moving" not in k}
        st = {k: v for k, v in p.items() if "moving" in k}
        z_ = fwd(x.to(dt)[:, None].repeat(1, 3, 1, 1), prm, training, st)
        om.keras_loss(z_, tgt.to(dt), "cce").backward()
        return z_, prm

    z64, p64 = oracle(torch.float64)
    _, p32 = oracle(torch.float32)
    from acfe import ops

    z = m(x.to(dtype).to(cuda))
    _, dz = ops.loss_and_grad(z, tgt.float().to(cuda), "cce")
    z.backward(dz)
    print(f"logits rel {t.rel(z, z64):.3e}")
    names = [n for n, _ in m.named_parameters()]
    g_dev = torch.cat([q.grad.reshape(-1).double().cpu() for q in m.parameters()])
    g64 = torch.cat([p64[n].grad.reshape(-1) for n in names])
    g32 = torch.cat([p32[n].grad.reshape(-1) for n in names])
    print(f"arena dev {t.rel(g_dev, g64):.3e}  e32 {t.rel(g32, g64):.3e}")
    for n, q in m.named_parameters():
        ref = p64[n].grad
        print(f"{n:40s} dev {t.rel(q.grad, ref):.3e}  e32 {t.rel(p32[n].grad, ref):.3e}  |ref| {ref.norm():.3e}")



def block_check(idx=1):
    """Run the whole bird model on the GPU (fp32, eval), capture block `idx`'s
    input and output gradient, and replay that block alone in the float64
    oracle with the SAME input / output gradient: isolates a block's backward."""
    import torch.nn.functional as F

    cuda = torch.device("cuda", 0)
    H, W, classes, N = 128, 64, 10, 2
    m = t._build("bird", (H, W, 3), classes, torch.float32, cuda)
    m.eval()
    cap = {}

    def fhook(mod, inp, out):
        cap["x"] = inp[0].detach().clone()
        z = out[0]
        z.register_hook(lambda g: cap.__setitem__("gz", g.detach().clone()))
        if inp[0].requires_grad:
            inp[0].register_hook(lambda g: cap.__setitem__("gx", g.detach().clone()))

    blk = m.blocks[idx]
    blk.register_forward_hook(fhook)
    x = t._input(N, H, W).float().to(cuda).requires_grad_(True)
    from acfe import ops

    tgt = torch.zeros(N, classes)
    tgt[0, 3] = tgt[1, 7] = 1
    z = m(x)
    _, dz = ops.loss_and_grad(z, tgt.to(cuda), "cce")
    z.backward(dz)
    p = {k: v.detach().double().cpu().clone().requires_grad_(True) for k, v in blk.state_dict().items()}
    X = cap["x"].double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    pre = ""
    Y = om.bn(X, p, "bn2a", False, relu=True, state=p)
    Y = om.conv(Y, p["conv21.weight"], p["conv21.bias"])
    Y = om.bn(Y, p, "bn2b", False, relu=True, state=p)
    Y = om.conv(Y, p["conv2b.weight"], p["conv2b.bias"])
    Z = F.relu(Y + X) if blk.relu_out else Y + X
    Z.backward(cap["gz"].double().cpu().permute(0, 3, 1, 2))
    print("block", idx, "replayed in float64 with the device's input and output gradient")
    print(f"  dx   rel {t.rel(cap['gx'].permute(0, 3, 1, 2), X.grad):.3e}" if "gx" in cap else "  (no dx)")
    for n, q in blk.named_parameters():
        print(f"  {n:24s} rel {t.rel(q.grad, p[n].grad):.3e}")


def block_steps(idx=1):
    """As block_check, then the block's ops one at a time on the GPU (unfused)
    against float64, comparing every intermediate gradient."""
    import torch.nn.functional as F
    from acfe import ops

    cuda = torch.device("cuda", 0)
    H, W, classes, N = 128, 64, 10, 2
    m = t._build("bird", (H, W, 3), classes, torch.float32, cuda)
    m.eval()
    cap = {}

    def fhook(mod, inp, out):
        cap["x"] = inp[0].detach().clone()
        out[0].register_hook(lambda g: cap.__setitem__("gz", g.detach().clone()))

    blk = m.blocks[idx]
    blk.register_forward_hook(fhook)
    tgt = torch.zeros(N, classes)
    tgt[0, 3] = tgt[1, 7] = 1
    with torch.no_grad():
        pass
    z = m(t._input(N, H, W).float().to(cuda))
    _, dz = ops.loss_and_grad(z, tgt.to(cuda), "cce")
    z.backward(dz)
    # device chain
    x = cap["x"].clone().requires_grad_(True)
    g = {}
    y1 = blk.bn2a(x, relu=True)
    u = blk.conv21(y1)
    y2 = blk.bn2b(u, relu=True)
    v = blk.conv2b(y2)
    zz = ops.add(v, x, relu=blk.relu_out)
    for nm, tt in (("y1", y1), ("u", u), ("y2", y2), ("v", v)):
        tt.register_hook(lambda gg, nm=nm: g.__setitem__(nm, gg.detach().clone()))
    zz.backward(cap["gz"])
    # float64 chain
    p = {k: v_.detach().double().cpu().clone().requires_grad_(True) for k, v_ in blk.state_dict().items()}
    X = cap["x"].double().cpu().permute(0, 3, 1, 2).requires_grad_(True)
    Y1 = om.bn(X, p, "bn2a", False, relu=True, state=p)
    U = om.conv(Y1, p["conv21.weight"], p["conv21.bias"])
    Y2 = om.bn(U, p, "bn2b", False, relu=True, state=p)
    V = om.conv(Y2, p["conv2b.weight"], p["conv2b.bias"])
    for T_ in (Y1, U, Y2, V):
        T_.retain_grad()
    Z = F.relu(V + X) if blk.relu_out else V + X
    Z.backward(cap["gz"].double().cpu().permute(0, 3, 1, 2))
    ref = {"y1": Y1, "u": U, "y2": Y2, "v": V}
    for nm in ("v", "y2", "u", "y1"):
        print(f"  grad {nm:3s} rel {t.rel(g[nm].permute(0, 3, 1, 2), ref[nm].grad):.3e}   "
              f"fwd rel {t.rel(dict(y1=y1, u=u, y2=y2, v=v)[nm].permute(0, 3, 1, 2), ref[nm]):.3e}")
    print(f"  grad x   rel {t.rel(x.grad.permute(0, 3, 1, 2), X.grad):.3e}")
    # relu mask agreement of bn2b and of the add
    pre = (u.detach() * 0)  # placeholder to keep shapes
    mask_dev = (y2 > 0).permute(0, 3, 1, 2).cpu()
    mask_ref = (Y2 > 0)
    print("  bn2b relu mask mismatches:", int((mask_dev != mask_ref).sum()), "of", mask_ref.numel())
    print("  y2 exact zeros dev/ref:", int((y2 == 0).sum()), int((Y2 == 0).sum()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "steps":
    block_steps(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    sys.exit(0)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "block":
    block_check(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    sys.exit(0)


if __name__ == "__main__":
    main()
