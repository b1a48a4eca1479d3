"""End-to-end parity of the two model families (HIP path) against the oracle
graphs of oracle/models.py (torch-CPU restatement of the Keras models).

Dropout is disabled (rate 0) so both sides are deterministic.

fp32 compute, eval-mode BN (well conditioned: e32 ~1e-6 for the bird model):
  rel-L2(logits) <= 1e-4; rel-L2(gradient arena) <= 1e-4; the MEDIAN
  per-parameter error <= max(4 x median e32, 1e-5); every parameter <= 5e-3.
  (e32 = error of the SAME oracle run in torch-CPU float32.)  A ReLU whose
  pre-activation lies within ~1e-7 of zero can take the other branch than in
  float64 -- at this size one element of 131072 in block 1's bn2b does -- and
  that alone moves the gradients upstream of it by up to ~1e-3, so the tight
  bound is put on the median, the loose one on every parameter.
fp32 compute, training-mode BN: rel-L2(logits) <= 1e-4; arena <= 4 x the
  arena e32; every parameter <= max(8 x e32, 4 x arena e32).  Tiny-batch
  training BatchNorm is ill-conditioned (arena e32 ~5e-3), so any change of
  summation order (e.g. BN statistics taken in the conv epilogue) lands at a
  few e32; gradients that are zero in exact arithmetic (biases of convs
  feeding a training-mode BN) must be ~0 absolutely.
bf16 compute, vs the oracle with the same bf16 storage points (storage="bf16"):
  eval-mode BN: rel-L2(logits) <= 1e-2, rel-L2(gradient arena) <= 5e-2
    (floor measured between fp32- and fp64-accumulating bf16 oracles:
     1.2e-3 / 8.8e-3);
  training-mode BN: a whole-model bf16 training step at init is chaotic (two
    bf16-storage oracles differ by 3.6 % in the logits and 61 % in the
    gradients at N = 2), so it is not checked whole with a loose bound; the
    benchmarked mode is checked at the T1 shape segment by segment with fixed
    bounds (test_bird_t1_shape_bf16_train_segments) and per residual block
    (test_block_bf16_train_fixed_bounds).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import models as om  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _build(kind, shape, classes, dtype, cuda):
    if kind == "bird":
        from resnet.wr_resnet_bird import WRResNet
    else:
        from resnet.wr_resnet import WRResNet
    torch.manual_seed(0)
    m = WRResNet(input_shape=shape, classes=classes, dtype=dtype, dropout=0.0).to(cuda)
    # non-trivial BN affine parameters so their gradients are exercised
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("gamma"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("beta") or name.endswith("bias"):
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
        for name, b in m.named_buffers():
            if name.endswith("moving_mean"):
                b.copy_(0.1 * torch.randn(b.shape, generator=g))
            elif name.endswith("moving_variance"):
                b.copy_(1 + 0.5 * torch.rand(b.shape, generator=g))
    return m


def _input(n, h, w, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((n, h, w), generator=g, dtype=torch.float64) * 2 - 1


# (the bf16 training-mode whole-model case is test_bird_t1_shape_bf16_train_segments:
# at the model level the bf16 emulation is itself 26 % (output) / 93 % (arena)
# from exact math at init, so only per-segment bounds can be fixed)
CASES = [("f32", True), ("f32", False), ("bf16", False)]


@pytest.mark.parametrize("kind", ["bird", "wrn"])
@pytest.mark.parametrize("prec,training", CASES, ids=["f32-train", "f32-eval", "bf16-eval"])
def test_model_step_parity(cuda, kind, prec, training):
    dtype = torch.float32 if prec == "f32" else torch.bfloat16
    H, W, classes, N = 128, 64, 10, 2
    m = _build(kind, (H, W, 3), classes, dtype, cuda)
    m.train(training)
    x = _input(N, H, W)
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).double()
    tgt = torch.zeros(N, classes, dtype=torch.float64)
    tgt[0, 3] = tgt[1, 7] = 1
    # oracle
    fwd = om.wr_resnet_bird if kind == "bird" else om.wr_resnet

    storage = "bf16" if dtype == torch.bfloat16 else None

    def oracle(dt, storage=storage):
        p = {k: v.detach().to(dt).cpu().clone() for k, v in m.state_dict().items()}
        prm = {k: v.requires_grad_(True) for k, v in p.items() if "moving" not in k}
        st = {k: v for k, v in p.items() if "moving" in k}
        z_ = fwd(x.to(dt)[:, None].repeat(1, 3, 1, 1), prm, training, st, storage=storage)
        l_ = om.keras_loss(z_, tgt.to(dt), "cce")
        l_.backward()
        return z_, l_, prm, st

    z_ref, loss_ref, params, state = oracle(torch.float64)
    _z32, _, params32, _ = oracle(torch.float32)
    # device
    from acfe import ops

    xd = x.to(dtype).to(cuda)
    z = m(xd)
    loss, dz = ops.loss_and_grad(z, tgt.float().to(cuda), "cce")
    z.backward(dz)
    lt = 1e-4 if dtype == torch.float32 else 1e-2
    assert torch.isfinite(z).all() and torch.isfinite(loss).all()
    assert rel(z, z_ref) < lt, (rel(z, z_ref), z, z_ref)
    assert abs(loss.item() - loss_ref.item()) < lt * max(1.0, abs(loss_ref.item()))
    names = [n for n, q in m.named_parameters()]
    g_dev = torch.cat([q.grad.reshape(-1).double().cpu() for q in m.parameters()])
    g_ref = torch.cat([params[n].grad.reshape(-1) for n in names])
    if dtype == torch.float32:
        gnorm = g_ref.norm().item()
        g32 = torch.cat([params32[n].grad.reshape(-1) for n in names])
        e32_arena = rel(g32, g_ref)
        assert rel(g_dev, g_ref) < (4 * e32_arena if training else 1e-4), (rel(g_dev, g_ref), e32_arena)
        devs, e32s = [], []
        for n, q in m.named_parameters():
            ref = params[n].grad
            if ref.norm().item() < 1e-9 * gnorm:  # exactly zero in exact arithmetic
                assert q.grad.double().norm().item() < 1e-5 * gnorm, n
                continue
            e32 = rel(params32[n].grad, ref)
            d = rel(q.grad, ref)
            devs.append(d)
            e32s.append(e32)
            bound = max(8 * e32, 4 * e32_arena) if training else 5e-3
            assert d < bound, (n, d, e32)
        if not training:
            med = sorted(devs)[len(devs) // 2]
            assert med < max(4 * sorted(e32s)[len(e32s) // 2], 1e-5), med
    else:
        assert rel(g_dev, g_ref) < 5e-2, rel(g_dev, g_ref)
    # moving statistics updated like Keras (momentum 0.99)
    for k, v in state.items():
        assert rel(m.state_dict()[k], v) < (1e-4 if dtype == torch.float32 else 3e-2), k


BLOCK_CASES = [("bird", 0, 8, 128, 128), ("bird", 1, 8, 128, 128), ("bird", 3, 8, 128, 128),
               ("wrn", 0, 4, 64, 64), ("wrn", 3, 4, 64, 64)]


@pytest.mark.parametrize("kind,bi,N,H,W", BLOCK_CASES,
                         ids=["bird-s1b0", "bird-s1b1", "bird-s2b0", "wrn-s1b0", "wrn-s2b0"])
def test_block_bf16_train_fixed_bounds(cuda, kind, bi, N, H, W):
    """bf16 training-mode residual blocks with FIXED bounds (VERDICT r02 next
    #1, the well-conditioned bf16 training case).

    A whole-model bf16 training step at init is not well conditioned at any
    batch size: the loss gradient reaching the pooled head is nearly uniform
    over pixels, so every training-mode BatchNormalization backward cancels it
    and what is left is bf16 rounding noise (two bf16-storage oracles, fp32 vs
    fp64 accumulation, differ by 63 % in their gradients at N = 16, 128 x 64;
    test_model_step_parity keeps that case with spread-relative bounds).  Here
    each block runs in training mode on a random bf16 input with a random
    per-pixel upstream gradient, which keeps the BN backward well conditioned.

    What remains is discrete: with bf16 storage a ReLU input or a 2x2 max-pool
    window that sits within a rounding step of its threshold / tie takes the
    other branch whenever two implementations round at different points, and
    each flip moves an O(1) gradient entry.  The bf16 emulation of the Keras
    storage points (oracle storage="bf16") is itself 5-11 % (input gradient)
    and 5-9 % (parameter arena) rel-L2 from exact float64 math on these
    blocks, and the device -- whose fused nodes keep some of those tensors in
    fp32 (the 1x1+BN node, the pooled / residual epilogues) -- lands at the
    same distance from exact.  Bounds: the forward output within 1e-2 of the
    bf16 oracle (rounding is the only difference there) and within 1.5e-2 of
    exact; input gradient and parameter arena within 0.14 / 0.12 of exact
    (1.3x the emulation's own worst case); BN moving statistics within 1e-2."""
    m = _build(kind, (H, W, 3), 10, torch.bfloat16, cuda)
    m.train(True)
    blk = m.blocks[bi]
    pre = f"blocks.{bi}."
    if kind == "bird":
        h, w, c = H, W // 2, 16
    else:
        h, w, c = H, W, 16
    for j in range(bi):
        b = m.blocks[j]
        h, w, c = -(-h // b.stride), -(-w // b.stride), b.out_channels
    g = torch.Generator().manual_seed(11)
    x = torch.randn((N, c, h, w), generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    dz = None

    def oracle(storage):
        nonlocal dz
        p = {k: v.detach().double().cpu().clone() for k, v in m.state_dict().items() if k.startswith(pre)}
        prm = {k: v.requires_grad_(True) for k, v in p.items() if "moving" not in k}
        st = {k: v for k, v in p.items() if "moving" in k}
        xr = x.clone().requires_grad_(True)
        if kind == "bird":
            z_ = om.bird_block(xr, prm, pre, blk.stride, blk.relu_out, True, st, storage=storage)
        else:
            z_ = om.wrn_block(xr, prm, pre, blk.stride, True, st, storage=storage)
        if dz is None:
            dz = torch.randn(z_.shape, generator=torch.Generator().manual_seed(12), dtype=torch.float64)
            dz = dz.to(torch.bfloat16).double()
        (z_ * dz).sum().backward()
        return z_.detach(), xr.grad, prm, st

    z_bf, dx_bf, prm_bf, st_bf = oracle("bf16")
    z_ex, dx_ex, prm_ex, _ = oracle(None)
    # device (NHWC)
    xd = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(cuda).requires_grad_(True)
    z, _ = blk(xd)
    z.backward(dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(cuda))
    names = [n for n, _ in blk.named_parameters()]
    g_dev = torch.cat([q.grad.reshape(-1).double().cpu() for q in blk.parameters()])
    g_bf = torch.cat([prm_bf[pre + n].grad.reshape(-1) for n in names])
    g_ex = torch.cat([prm_ex[pre + n].grad.reshape(-1) for n in names])
    zd, dxd = z.permute(0, 3, 1, 2), xd.grad.permute(0, 3, 1, 2)
    print(f"{kind} block {bi} bf16 train: out {rel(zd, z_bf):.2e} (emulation vs exact {rel(z_bf, z_ex):.2e}, "
          f"device vs exact {rel(zd, z_ex):.2e}); dx vs exact {rel(dxd, dx_ex):.2e} (emulation {rel(dx_bf, dx_ex):.2e}); "
          f"arena vs exact {rel(g_dev, g_ex):.2e} (emulation {rel(g_bf, g_ex):.2e})")
    assert rel(zd, z_bf) <= 1e-2
    assert rel(zd, z_ex) <= 1.5e-2
    assert rel(dxd, dx_ex) <= 0.14
    assert rel(g_dev, g_ex) <= 0.12
    sd = blk.state_dict()
    for k, v in st_bf.items():
        assert rel(sd[k[len(pre):]], v) <= 1e-2, k


def test_bird_shapes_reference_config(cuda):
    """The T1 configuration: 128 mels x 513 frames x 3, 50 classes."""
    from resnet.wr_resnet_bird import WRResNet, flops_per_clip

    m = WRResNet(input_shape=(128, 513, 3), classes=50)
    assert m.feature_hw == (16, 32)
    assert m.prediction.kernel.shape == (32, 50)
    assert [tuple(b.conv21.weight.shape[:1]) for b in m.blocks] == [(128,), (64,), (64,), (64,), (32,), (32,),
                                                                     (32,), (16,), (16,)]
    n = sum(p.numel() for p in m.parameters())
    assert 2.2e6 < n < 2.4e6, n
    assert abs(flops_per_clip(m) / 1e9 - 16.91) < 0.05


@pytest.mark.parametrize("kind", ["bird", "wrn"])
@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
def test_arena_gradients_match_autograd(cuda, kind, training):
    """Parameters in a ParamArena get their conv-weight, conv-bias and BN
    gamma/beta gradients accumulated in place by the producing kernels (beta 1
    into the zeroed arena, autograd sees None): bit-identical to the gradients
    autograd assigns without the arena, and a second backward without
    zero_grad accumulates (2x)."""
    from acfe import ops
    from acfe.layers import ParamArena

    H, W, classes, N = 128, 64, 10, 2
    tgt = torch.zeros(N, classes, device=cuda)
    tgt[0, 3] = tgt[1, 7] = 1
    x = _input(N, H, W).to(torch.bfloat16).to(cuda)
    grads = []
    for use_arena in (False, True):
        m = _build(kind, (H, W, 3), classes, torch.bfloat16, cuda)
        m.train(training)
        arena = ParamArena(m, cuda) if use_arena else None
        if arena is not None:
            arena.zero_grad()
        z = m(x)
        _, dz = ops.loss_and_grad(z, tgt, "cce")
        z.backward(dz)
        grads.append([p.grad.detach().clone() for p in m.parameters()])
        if arena is not None:
            z = m(x)
            _, dz = ops.loss_and_grad(z, tgt, "cce")
            z.backward(dz)
            again = [p.grad.detach().clone() for p in m.parameters()]
    names = [n for n, _ in m.named_parameters()]
    for n, a, b in zip(names, grads[0], grads[1]):
        assert torch.equal(a, b), (n, rel(b, a))
    for n, a, b in zip(names, grads[1], again):
        if not training:  # training-mode BN statistics move between the two forwards
            torch.testing.assert_close(b, 2 * a, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("kind", ["bird", "wrn"])
def test_weight_packer_matches_per_call_packing(cuda, kind):
    """Trainer packs every conv weight of a step with ONE launch
    (acfe_conv2d_pack_weights_batch) from the second step on: each packed form
    is bit-identical to acfe_conv2d_pack_weights of the same weight, the
    packer covers both orientations of every arena conv weight the step used,
    and a step with the packer gives the same loss as a step without."""
    from acfe import ops
    from acfe.train import FrontEnd, Trainer

    H, W, classes, N = 128, 513, 10, 2
    m = _build(kind, (H, W, 3), classes, torch.bfloat16, cuda)
    fe = FrontEnd(n_mels=H, dtype=torch.bfloat16, device=cuda, pcen=False).to(cuda)
    tr = Trainer(m, fe, lr=0.0, loss="cce", device=cuda)
    g = torch.Generator().manual_seed(5)
    x = torch.randn((N, 144000), generator=g).clamp(-1, 1).to(cuda)
    y = torch.zeros(N, classes, device=cuda)
    y[0, 1] = y[1, 2] = 1
    l1, _ = tr.step(x, y)
    assert tr.packer is not None
    flips = {(e[0].data_ptr(), e[2]) for e in tr.packer.entries}
    convs = [p for n, p in m.named_parameters() if p.dim() == 4 and n.endswith("weight")]
    assert len(tr.packer.entries) >= len(convs)
    outs = tr.packer.pack()
    for w, dtype, flip, key in tr.packer.entries:
        ops._PACK_ACTIVE = None
        ref = ops.pack_weights(w, dtype, flip)
        assert torch.equal(outs[key], ref), (tuple(w.shape), flip)
    l2, _ = tr.step(x, y)  # lr 0: same weights, packed by the batch kernel now
    torch.cuda.synchronize()
    assert abs(float(l2) - float(l1)) <= 1e-5 * max(1.0, abs(float(l1)))
    assert len(flips) == len(tr.packer.entries)


def test_bird_t1_shape_bf16_train_segments(cuda):
    """The benchmarked mode whole: wr_resnet_bird in bf16 with training-mode
    BatchNormalization at the T1 shape (128 x 513, 50 classes, N = 4 clips),
    a random per-pixel upstream gradient injected at the head maps
    (conv2d_head_3's output, before the logmeanexp poolings) so every BN
    backward stays conditioned, every segment of the device's own chain held to
    FIXED bounds.

    Chained end to end, no bf16 implementation can be held to a fixed bound
    here: rounding at the storage points compounds ~1.3x per block and the
    final BN doubles it, so the bf16-storage emulation itself lands 26 %
    (head maps) and 93 % (gradient arena) rel-L2 from exact float64 math at
    init, and two emulations (f32 / f64 accumulation) differ by 13 % / 66 %
    (oracle dry run at this shape).  Each segment is therefore checked on the
    device's own input and upstream gradient (teacher forcing): the stem
    (conv1_1 + BN + MaxPool2D(1, 2)), the nine residual blocks and the head
    (final_bn .. conv2d_head_3), each against the bf16-storage oracle and exact
    float64 math of the same segment.  Bounds (the block test's): segment
    output <= 1e-2 of the emulation and <= 1.5e-2 of exact; input gradient
    <= 0.14 and parameter gradients <= 0.12 of exact (the emulation itself:
    <= 9.6e-2 / 7.7e-2 on these segments)."""
    import torch.nn.functional as F

    H, W, classes, N = 128, 513, 50, 4
    m = _build("bird", (H, W, 3), classes, torch.bfloat16, cuda)
    m.train(True)
    sd = {k: v.detach().double().cpu().clone() for k, v in m.state_dict().items()}
    x = _input(N, H, W, seed=5).to(torch.bfloat16).double()
    # device forward with each block's input / output and their gradients captured
    cap = {}

    def pre_hook(i):
        def f(mod, args):
            cap[f"in{i}"] = args[0]
            if i == 0:
                args[0].register_hook(lambda g: cap.__setitem__("gin0", g))
        return f

    def post_hook(i):
        def f(mod, args, out):
            z = out[0]
            cap[f"in{i + 1}"] = z
            z.register_hook(lambda g: cap.__setitem__(f"gin{i + 1}", g))
        return f

    hs = []
    for i, blk in enumerate(m.blocks):
        hs.append(blk.register_forward_pre_hook(pre_hook(i)))
        hs.append(blk.register_forward_hook(post_hook(i)))
    xd = x.to(torch.bfloat16).to(cuda).requires_grad_(False)
    zmap = m.head_maps(xd)  # [N, h, w, classes]
    dz = torch.randn((N, classes) + tuple(zmap.shape[1:3]), generator=torch.Generator().manual_seed(12),
                     dtype=torch.float64).to(torch.bfloat16).double()
    zmap.backward(dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(cuda))
    torch.cuda.synchronize()
    for h in hs:
        h.remove()
    dev_grads = {n: q.grad.detach().double().cpu() for n, q in m.named_parameters() if q.grad is not None}
    nchw = lambda t: t.detach().double().cpu().permute(0, 3, 1, 2)  # noqa: E731

    def seg(kind, i, xin, gout, storage):
        p = {k: v.clone().requires_grad_("moving" not in k) for k, v in sd.items()}
        xr = xin.clone().requires_grad_(True)
        if kind == "stem":
            z = om.conv(xr[:, None].repeat(1, 3, 1, 1), p["conv1_1.weight"], p["conv1_1.bias"], storage=storage)
            z = om.bn(z, p, "bn_stem", True, storage=storage)
            z = F.max_pool2d(z, (1, 2), (1, 2))
            pre = ("conv1_1.", "bn_stem.")
        elif kind == "block":
            blk = m.blocks[i]
            z = om.bird_block(xr, p, f"blocks.{i}.", blk.stride, blk.relu_out, True, None, storage=storage)
            pre = (f"blocks.{i}.",)
        else:
            z = om.bn(xr, p, "final_bn", True, relu=True, storage=storage)
            for c, b in (("head_conv1", "head_bn1"), ("head_conv2", "head_bn2")):
                z = om.conv(z, p[c + ".weight"], p[c + ".bias"], storage=storage)
                z = om.bn(z, p, b, True, storage=storage)
            z = om.conv(z, p["head_conv3.weight"], p["head_conv3.bias"], storage=storage)
            pre = ("final_bn.", "head_")
        (z * gout).sum().backward()
        names = [k for k in p if k.startswith(pre) and "moving" not in k]
        return z.detach(), xr.grad, names, torch.cat([p[k].grad.reshape(-1) for k in names])

    segments = [("stem", 0, x, nchw(cap["gin0"]), nchw(cap["in0"]))]
    segments += [("block", i, nchw(cap[f"in{i}"]), nchw(cap[f"gin{i + 1}"]), nchw(cap[f"in{i + 1}"]))
                 for i in range(len(m.blocks))]
    segments += [("head", 0, nchw(cap[f"in{len(m.blocks)}"]), dz, nchw(zmap))]
    gin = {0: None}
    gin.update({i: nchw(cap[f"gin{i}"]) for i in range(len(m.blocks) + 1)})
    for kind, i, xin, gout, zdev in segments:
        z_bf, dx_bf, names, g_bf = seg(kind, i, xin, gout, "bf16")
        z_ex, dx_ex, _, g_ex = seg(kind, i, xin, gout, None)
        g_dev = torch.cat([dev_grads[k].reshape(-1) for k in names])
        tag = f"{kind} {i}"
        print(f"{tag}: out {rel(zdev, z_bf):.2e} / exact {rel(zdev, z_ex):.2e}; arena {rel(g_dev, g_ex):.2e} "
              f"(emulation {rel(g_bf, g_ex):.2e})", end="")
        assert rel(zdev, z_bf) <= 1e-2, tag
        assert rel(zdev, z_ex) <= 1.5e-2, tag
        assert rel(g_dev, g_ex) <= 0.12, tag
        if kind != "stem":  # the input gradient the device delivered to this segment's input
            k = len(m.blocks) if kind == "head" else i
            dx_dev = gin[k]
            # a ReLU output as input: the consumer BN folds that ReLU's backward,
            # so the device delivers the gradient masked by [x > 0]
            relu_in = kind == "head" or (i > 0 and m.blocks[i - 1].relu_out)
            mask = (xin > 0).double() if relu_in else torch.ones_like(xin)
            print(f"; dx {rel(dx_dev * mask, dx_ex * mask):.2e} (emulation {rel(dx_bf * mask, dx_ex * mask):.2e})")
            assert rel(dx_dev * mask, dx_ex * mask) <= 0.14, tag
        else:
            print()
