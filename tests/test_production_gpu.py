"""Oracle parity of the T1 hot kernels at the shapes and tile / split counts
they run at in the training step.

The dominant stage-1 block-0 layers of wr_resnet_bird at 128 mels x 513
frames (resnet/wr_resnet_bird.py:136-178):
  * conv21 3x3 128->128 @ 128x256 -> MaxPool2D(2) -> Dropout -> BN sums
    (acfe_conv2d_fwd_pool, k_conv3x3_rows<128,6,1>)
  * its backward: acfe_conv2d_dgrad_unpool (k_conv3x3_rows<128,6,2>) and
    acfe_conv2d_wgrad_unpool (k_wgrad3x3_halo<128,true>, split-K + combine)
  * conv2b 3x3 64->64 @ 64x128 + residual Add (+ReLU) + BN sums
    (acfe_conv2d_fwd_add, k_conv3x3_rows<64,6,3>)
at N = 8 / 32 clips, i.e. 704 output tiles for the 256 persistent workgroups
(every workgroup walks several tiles, the inter-tile pipeline runs) and the
production split-K counts of the weight gradient.

The oracle is torch-CPU float64 convolution of the same bf16 operands
(oracle.models.conv semantics: Keras "same" = pad 1 for 3x3).  Bounds:
  * bf16 outputs (y, dx): |gpu - exact| <= 1 bf16 ulp(exact) + 1e-4 -- the
    kernel accumulates in fp32 and rounds once, so its error is half an ulp
    plus fp32 accumulation noise; a wrong tap, channel or tile is off by O(1);
  * pooled output: the same bound against max over the 2x2 window of the
    exact conv (rounding is monotone, so max and round commute), and the
    argmax byte must point at a value within that bound of the window max;
  * weight gradient (fp32 out): rel-L2 <= 5e-5 and every element within
    5e-4 x max|exact| (fp32 accumulation over 131072-262144 pixels);
  * BN statistics slabs: the float64 sums of the stored output to rel 1e-6
    (the epilogue sums each wave's 16-row fragment in fp32 first).
"""
import itertools

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
F64 = torch.float64


@pytest.fixture(scope="module")
def env(cuda):
    from acfe import ops
    from acfe._lib import call, lib
    from acfe._torch import ptr, stream

    return ops, call, lib, ptr, stream


def _ulp(t):
    """bf16 unit in the last place of each element of t (float64)."""
    e = torch.floor(torch.log2(t.abs().clamp_min(2.0 ** -120)))
    return torch.pow(2.0, e - 7)


def _within_ulp(gpu, exact, atol=1e-4, what="", extra=0.0):
    g = gpu.detach().to(F64).cpu()
    err = (g - exact).abs()
    bad = err > _ulp(exact) + atol + extra
    nbad = int(bad.sum())
    assert nbad == 0, (what, nbad, float(err.max()), float((err / (_ulp(exact) + atol)).max()))


def _oracle_conv(x_nhwc, w_krsc, b=None):
    """exact 'same' 3x3 conv of bf16 operands: x [N,H,W,C] bf16, w fp32 KRSC
    (the kernel multiplies its bf16 packing) -> [N,H,W,K] float64."""
    x = x_nhwc.detach().cpu().to(F64).permute(0, 3, 1, 2)
    w = w_krsc.detach().cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    y = F.conv2d(x, w, None if b is None else b.detach().cpu().to(F64), padding=1)
    return y.permute(0, 2, 3, 1).contiguous()


def _sums(t):
    t = t.detach().to(F64).cpu().reshape(-1, t.shape[-1])
    return torch.stack([t.sum(0), (t * t).sum(0)])


def _data(N, H, W, C, K, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn((N, H, W, C), generator=g).to(BF)
    w = torch.randn((K, 3, 3, C), generator=g) * (1.0 / (3 * C ** 0.5))
    b = torch.randn((K,), generator=g) * 0.1
    return x.to(device), w.to(device), b.to(device), g


def test_conv_fwd_pool_production(env, cuda):
    """acfe_conv2d_fwd_pool at the T1 stage-1 shape (8 clips x 128 x 256,
    128 -> 128): pooled values, argmax bytes, dropout mask and BN sums."""
    ops, call, lib, ptr, stream = env
    N, H, W, C, K = 8, 128, 256, 128, 128
    assert lib.acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, 1)
    x, w, b, g = _data(N, H, W, C, K, 101, cuda)
    wp = ops.pack_weights(w, BF, False)
    P, Q = H // 2, W // 2
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    y0 = torch.empty((N, P, Q, K), dtype=BF, device=cuda)
    am0 = torch.empty((N, P, Q, K), dtype=torch.uint8, device=cuda)
    st0 = torch.empty((rows, 2, wp.shape[0]), dtype=F64, device=cuda)
    call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y0), ptr(am0), 0.0, 0, ptr(st0),
         1, stream())
    y1, am1 = torch.empty_like(y0), torch.empty_like(am0)
    st1 = torch.empty_like(st0)
    call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y1), ptr(am1), 0.1, 4242,
         ptr(st1), 1, stream())
    torch.cuda.synchronize()
    exact = _oracle_conv(x, w, b)                                   # [N, H, W, K]
    win = exact.reshape(N, P, 2, Q, 2, K).permute(0, 1, 3, 5, 2, 4).reshape(N, P, Q, K, 4)
    wmax = win.max(-1).values
    _within_ulp(y0, wmax, what="pooled")
    # the argmax byte names a (near-)maximum of the window: a*2+b in [0, 4)
    am = am0.cpu().long()
    assert int(am.max()) < 4
    picked = torch.gather(win, -1, am[..., None])[..., 0]
    assert bool(((wmax - picked) <= _ulp(wmax) + 1e-4).all())
    # dropout: the same pooled values with acfe_dropout's mask, same argmax
    ref = torch.empty_like(y0)
    call("acfe_dropout", ptr(y0), y0.numel(), 0.1, 4242, ptr(ref), 1, stream())
    assert torch.equal(y1, ref) and torch.equal(am1, am0)
    # BN sums of the stored (dropped-out) output
    torch.testing.assert_close(st1.sum(0)[:, :K].cpu(), _sums(y1), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("N,H,W,C,K", [(8, 128, 256, 128, 128), (16, 64, 128, 128, 64)], ids=["s1b0", "s2b0"])
def test_conv_unpool_backward_production(env, cuda, N, H, W, C, K):
    """acfe_conv2d_dgrad_unpool / acfe_conv2d_wgrad_unpool at the T1 stage-1
    shape and the stage-2 branch21 (128 -> 64 @ 64x128; its weight gradient on
    the two-rows-per-step halo kernel) from a pooled gradient and argmax bytes:
    dX and dW against the float64 gradients of the exact convolution of the
    expanded (unpooled) gradient."""
    ops, call, lib, ptr, stream = env
    x, w, b, g = _data(N, H, W, C, K, 102, cuda)
    P, Q = H // 2, W // 2
    gp = (torch.randn((N, P, Q, K), generator=g) * 0.5).to(BF)
    am = torch.randint(0, 4, (N, P, Q, K), generator=g, dtype=torch.uint8)
    # expanded gradient: gp at (2p + a, 2q + b) with a*2+b = argmax
    onehot = F.one_hot(am.long(), 4).to(F64).reshape(N, P, Q, K, 2, 2).permute(0, 1, 4, 2, 5, 3)
    full = (onehot * gp.to(F64)[:, :, None, :, None, :]).reshape(N, H, W, K)
    gp, am = gp.to(cuda), am.to(cuda)
    wf = ops.pack_weights(w, BF, True)
    dx = torch.empty((N, H, W, C), dtype=BF, device=cuda)
    call("acfe_conv2d_dgrad_unpool", ptr(gp), ptr(am), N, H, W, K, ptr(wf), C, 1, 1, ptr(dx), 1, stream())
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw = torch.full((K, 3, 3, C), 0.25, device=cuda)  # beta 1: accumulated onto
    call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(gp), ptr(am), K, 1, 1, ptr(dw), 1.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    wd = w.detach().cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gfull = full.permute(0, 3, 1, 2)
    dx_exact = F.conv_transpose2d(gfull, wd, padding=1).permute(0, 2, 3, 1)
    _within_ulp(dx, dx_exact, what="dgrad_unpool")
    xd = x.cpu().to(F64).permute(0, 3, 1, 2)
    dw_exact = torch.nn.grad.conv2d_weight(xd, wd.shape, gfull, padding=1).permute(0, 2, 3, 1) + 0.25
    d = dw.cpu().to(F64)
    assert ((d - dw_exact).norm() / dw_exact.norm()).item() < 5e-5
    assert ((d - dw_exact).abs().max() / dw_exact.abs().max()).item() < 5e-4


@pytest.mark.parametrize("relu,shape", [(False, (32, 64, 128, 64, 64)), (True, (32, 64, 128, 64, 64)),
                                        (True, (32, 32, 64, 32, 128)), (False, (8, 13, 70, 32, 128)),
                                        (True, (32, 16, 32, 16, 256)), (False, (8, 13, 70, 16, 256))],
                         ids=["rows", "rows-relu", "c32-relu", "c32-ragged", "c16-256-relu", "c16-256-ragged"])
def test_conv_fwd_add_production(env, cuda, relu, shape):
    """acfe_conv2d_fwd_add at the stage-1 conv2b shape (64x128, 64 -> 64) for 32
    clips and at wr_resnet_bird's stage-2 / 3 branch2b (32 -> 128 at 32 x 64,
    16 -> 256 at 16 x 32, k_conv3x3_cw; ragged images): (ReLU)(conv + bias + shortcut) within one
    ulp of the exact value of the bf16 sum, BN sums of the stored output."""
    ops, call, lib, ptr, stream = env
    N, H, W, C, K = shape
    assert lib.acfe_conv2d_fwd_add_supported(N, H, W, C, K, 1)
    x, w, b, g = _data(N, H, W, C, K, 103 + relu, cuda)
    sc = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    wp = ops.pack_weights(w, BF, False)
    z = torch.empty((N, H, W, K), dtype=BF, device=cuda)
    st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=F64, device=cuda)
    call("acfe_conv2d_fwd_add", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(sc), int(relu), ptr(z), ptr(st), 1,
         stream())
    torch.cuda.synchronize()
    conv = _oracle_conv(x, w, b)
    exact = conv + sc.cpu().to(F64)
    if relu:
        exact = exact.clamp_min(0)
    # the conv output is rounded to bf16 before the Add (conv2d -> add), so a
    # cancelling sum may carry half an ulp of the conv value on top
    _within_ulp(z, exact, what="fwd_add", extra=0.5 * _ulp(conv))
    torch.testing.assert_close(st.sum(0)[:, :K].cpu(), _sums(z), rtol=1e-6, atol=1e-6)


def test_conv_rows_dgrad_wgrad_production(env, cuda):
    """The un-pooled stride-1 3x3 128->64 (stage-1 block-0 conv2b at 64x128 with
    128 input channels) dgrad and wgrad for 16 clips against float64."""
    ops, call, lib, ptr, stream = env
    N, H, W, C, K = 16, 64, 128, 128, 64
    x, w, b, g = _data(N, H, W, C, K, 105, cuda)
    dy = (torch.randn((N, H, W, K), generator=g) * 0.5).to(BF).to(cuda)
    wf = ops.pack_weights(w, BF, True)
    dx = torch.empty((N, H, W, C), dtype=BF, device=cuda)
    call("acfe_conv2d_dgrad", ptr(dy), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx), 1, None, stream())
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw = torch.empty((K, 3, 3, C), device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    wd = w.cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    _within_ulp(dx, F.conv_transpose2d(gd, wd, padding=1).permute(0, 2, 3, 1), what="dgrad")
    dw_exact = torch.nn.grad.conv2d_weight(x.cpu().to(F64).permute(0, 3, 1, 2), wd.shape, gd,
                                           padding=1).permute(0, 2, 3, 1)
    d = dw.cpu().to(F64)
    assert ((d - dw_exact).norm() / dw_exact.norm()).item() < 5e-5
    assert ((d - dw_exact).abs().max() / dw_exact.abs().max()).item() < 5e-4


@pytest.mark.parametrize("H,W,C,K,R,st", [(128, 513, 64, 128, 3, 2), (64, 257, 128, 256, 3, 3),
                                          (128, 513, 64, 128, 1, 2), (64, 257, 128, 256, 1, 3)],
                         ids=["s2b0_conv2a", "s3b0_conv2a", "s2b0_shortcut", "s3b0_shortcut"])
def test_strided_dgrad_wr_resnet_production(env, cuda, H, W, C, K, R, st):
    """wr_resnet's strided layers (resnet/wr_resnet.py:22, stage-2/3 block-0
    conv2a 3x3 and the 1x1 shortcuts at strides 2 and 3, TF "same" / "valid"
    padding) at the T1/I input 128 x 513: the sub-pixel phase dgrad against
    the float64 transposed convolution of the same bf16 operands, every
    element within one bf16 ulp + 1e-4."""
    ops, call, lib, ptr, stream = env
    N = 2
    g = torch.Generator(device="cpu").manual_seed(7 + st + R)
    w = (torch.randn((K, R, R, C), generator=g) * (1.0 / (R * C ** 0.5))).to(cuda)
    if R == 3:
        P, pt = ops.same_padding(H, 3, st)
        Q, pl = ops.same_padding(W, 3, st)
    else:
        P, Q, pt, pl = ops.valid_out(H, 1, st), ops.valid_out(W, 1, st), 0, 0
    dy = (torch.randn((N, P, Q, K), generator=g) * 0.5).to(BF).to(cuda)
    wf = ops.pack_weights(w, BF, True)
    dx = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    nb = lib.acfe_conv2d_dgrad_workspace(N, P, Q, K, C, R, R, st, pt, pl, H, W, 1)
    ws = torch.empty((nb,), dtype=torch.uint8, device=cuda)
    call("acfe_conv2d_dgrad", ptr(dy), N, P, Q, K, ptr(wf), C, R, R, st, pt, pl, H, W, ptr(dx), 1, ptr(ws), stream())
    torch.cuda.synchronize()
    wd = w.cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    # exact dX: the adjoint of the padded strided conv, cropped to H x W
    xr = torch.zeros((N, C, H, W), dtype=F64, requires_grad=True)
    xp = F.pad(xr, (pl, max(0, (Q - 1) * st + R - W - pl), pt, max(0, (P - 1) * st + R - H - pt)))
    (F.conv2d(xp, wd, stride=st) * gd).sum().backward()
    assert torch.isfinite(dx.float()).all()
    _within_ulp(dx, xr.grad.permute(0, 2, 3, 1), what="strided dgrad")


# Randomised strided-dgrad sweep: the super-pixel GEMM (bf16, K % 64 == 0,
# C a power of two) and the phase fallback (C = 48, 96) at "same" / "valid"
# padding, strides 2 / 3, 3x3 / 1x1 / 2x2 / 5x5 filters, odd and even sizes
_S2D_SWEEP = [
    # N, H, W, C, K, R, st, padding
    (2, 17, 30, 64, 128, 3, 2, "same"), (1, 30, 17, 32, 64, 3, 2, "valid"), (2, 25, 26, 128, 64, 3, 3, "same"),
    (1, 19, 40, 16, 128, 3, 3, "valid"), (2, 16, 21, 64, 64, 1, 2, "valid"), (1, 23, 24, 128, 256, 1, 3, "valid"),
    (2, 14, 18, 64, 64, 2, 2, "same"), (1, 21, 22, 32, 128, 5, 2, "same"), (1, 20, 33, 64, 128, 5, 3, "same"),
    (2, 15, 19, 48, 64, 3, 2, "same"), (1, 18, 20, 96, 128, 3, 3, "same"), (2, 4, 5, 64, 64, 3, 2, "same"),
    # stride 4 takes the super-pixel GEMM; stride 5 must fall back to the
    # phase path (its block-row multiply is not exact: ADVICE r05)
    (2, 21, 26, 64, 64, 3, 4, "same"), (1, 17, 23, 64, 64, 3, 4, "valid"), (2, 26, 27, 64, 64, 3, 5, "same"),
    (1, 23, 31, 64, 64, 5, 5, "valid"),
]


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad", _S2D_SWEEP, ids=lambda v: str(v))
def test_strided_dgrad_sweep(env, cuda, N, H, W, C, K, R, st, pad):
    """acfe_conv2d_dgrad at stride 2 / 3 against the float64 adjoint of the
    padded strided conv of the same bf16 operands: every element within one
    bf16 ulp + 1e-4, every pixel written (the tap-less positions as zeros)."""
    ops, call, lib, ptr, stream = env
    g = torch.Generator(device="cpu").manual_seed(H * 131 + W * 7 + C + K + R + st)
    w = (torch.randn((K, R, R, C), generator=g) * (1.0 / (R * C ** 0.5))).to(cuda)
    if pad == "same":
        P, pt = ops.same_padding(H, R, st)
        Q, pl = ops.same_padding(W, R, st)
    else:
        P, Q, pt, pl = ops.valid_out(H, R, st), ops.valid_out(W, R, st), 0, 0
    dy = (torch.randn((N, P, Q, K), generator=g) * 0.5).to(BF).to(cuda)
    wf = ops.pack_weights(w, BF, True)
    dx = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    nb = lib.acfe_conv2d_dgrad_workspace(N, P, Q, K, C, R, R, st, pt, pl, H, W, 1)
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=cuda)
    call("acfe_conv2d_dgrad", ptr(dy), N, P, Q, K, ptr(wf), C, R, R, st, pt, pl, H, W, ptr(dx), 1, ptr(ws), stream())
    torch.cuda.synchronize()
    wd = w.cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    xr = torch.zeros((N, C, H, W), dtype=F64, requires_grad=True)
    xp = F.pad(xr, (pl, max(0, (Q - 1) * st + R - W - pl), pt, max(0, (P - 1) * st + R - H - pt)))
    (F.conv2d(xp, wd, stride=st) * gd).sum().backward()
    assert torch.isfinite(dx.float()).all()
    _within_ulp(dx, xr.grad.permute(0, 2, 3, 1), what="strided dgrad sweep")


def test_bird_t1_shape_eval_parity(cuda):
    """wr_resnet_bird at the T1 input (128 mels x 513 frames, 50 classes), bf16,
    eval-mode BN, 2 clips, against the bf16-storage float64 oracle
    (oracle.models.wr_resnet_bird): at this width stage 1 is 256 px wide, so
    the rows / pool / add / halo kernels all run inside the model.  Bounds as
    tests/test_model_gpu.py's bf16-eval case: logits <= 1e-2, gradient arena
    <= 5e-2 (oracle-vs-oracle floor f32/f64 accumulation ~1e-3 / 1e-2)."""
    from oracle import models as om
    from resnet.wr_resnet_bird import WRResNet
    from acfe import ops

    H, W, classes, N = 128, 513, 50, 2
    torch.manual_seed(0)
    m = WRResNet(input_shape=(H, W, 3), classes=classes, dtype=BF, dropout=0.0).to(cuda)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("gamma"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g))
            elif name.endswith("beta") or name.endswith("bias"):
                p.copy_(0.05 * torch.randn(p.shape, generator=g))
        for name, bb in m.named_buffers():
            if name.endswith("moving_mean"):
                bb.copy_(0.1 * torch.randn(bb.shape, generator=g))
            elif name.endswith("moving_variance"):
                bb.copy_(1 + 0.5 * torch.rand(bb.shape, generator=g))
    m.eval()
    x = (torch.rand((N, H, W), generator=g, dtype=F64) * 2 - 1).to(BF).double()
    tgt = torch.zeros(N, classes, dtype=F64)
    tgt[0, 3] = tgt[1, 41] = 1
    p = {k: v.detach().to(F64).cpu().clone() for k, v in m.state_dict().items()}
    prm = {k: v.requires_grad_(True) for k, v in p.items() if "moving" not in k}
    st = {k: v for k, v in p.items() if "moving" in k}
    z_ref = om.wr_resnet_bird(x[:, None].repeat(1, 3, 1, 1), prm, False, st, storage="bf16")
    om.keras_loss(z_ref, tgt, "cce").backward()
    z = m(x.to(BF).to(cuda))
    _, dz = ops.loss_and_grad(z, tgt.float().to(cuda), "cce")
    z.backward(dz)
    zr = z.detach().double().cpu()
    assert ((zr - z_ref.detach()).norm() / z_ref.detach().norm()).item() < 1e-2
    names = [n for n, _ in m.named_parameters()]
    g_dev = torch.cat([q.grad.reshape(-1).double().cpu() for q in m.parameters()])
    g_ref = torch.cat([prm[n].grad.reshape(-1) for n in names])
    assert ((g_dev - g_ref).norm() / g_ref.norm()).item() < 5e-2


@pytest.mark.parametrize("W,H,C,K", [(130, 20, 64, 64), (513, 20, 64, 64), (130, 22, 128, 128), (513, 10, 128, 128)],
                         ids=["W130", "W513", "W130k128", "W513k128"])
def test_conv_rows_partial_column_tile(env, cuda, W, H, C, K):
    """wr_resnet's 513- / 257-wide stages run the rows / halo kernels with a
    partial last 64-pixel column tile (masked loads past Q, masked stores):
    fwd (+ BN sums), stride-1 dgrad and wgrad through the generic entry points
    against float64, and the pooled forward at an even width.  K = C = 128:
    the one-wave k_conv3x3_1w<0> (fwd with BN sums, dgrad without), H = 22 /
    10: a partial last 4-row tile."""
    ops, call, lib, ptr, stream = env
    N = 4
    x, w, b, g = _data(N, H, W, C, K, 107, cuda)
    assert lib.acfe_conv2d_rows_supported(N, H, W, C, K, 3, 3, 1)
    wp, wf = ops.pack_weights(w, BF, False), ops.pack_weights(w, BF, True)
    y = torch.empty((N, H, W, K), dtype=BF, device=cuda)
    st = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=F64, device=cuda)
    call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y), 1, ptr(st), stream())
    dy = (torch.randn((N, H, W, K), generator=g) * 0.5).to(BF).to(cuda)
    dx = torch.empty_like(x)
    call("acfe_conv2d_dgrad", ptr(dy), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx), 1, None, stream())
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw = torch.empty((K, 3, 3, C), device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    _within_ulp(y, _oracle_conv(x, w, b), what="fwd partial")
    torch.testing.assert_close(st.sum(0)[:, :K].cpu(), _sums(y), rtol=1e-6, atol=1e-6)
    wd = w.cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    _within_ulp(dx, F.conv_transpose2d(gd, wd, padding=1).permute(0, 2, 3, 1), what="dgrad partial")
    dw_exact = torch.nn.grad.conv2d_weight(x.cpu().to(F64).permute(0, 3, 1, 2), wd.shape, gd,
                                           padding=1).permute(0, 2, 3, 1)
    d = dw.cpu().to(F64)
    assert ((d - dw_exact).norm() / dw_exact.norm()).item() < 5e-5
    if W % 2 == 0:
        assert lib.acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, 1)
        P, Q = H // 2, W // 2
        yp = torch.empty((N, P, Q, K), dtype=BF, device=cuda)
        am = torch.empty((N, P, Q, K), dtype=torch.uint8, device=cuda)
        call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(yp), ptr(am), 0.0, 0, None,
             1, stream())
        torch.cuda.synchronize()
        win = _oracle_conv(x, w, b).reshape(N, P, 2, Q, 2, K).permute(0, 1, 3, 5, 2, 4).reshape(N, P, Q, K, 4)
        _within_ulp(yp, win.max(-1).values, what="pool partial")


def test_conv_rows_narrow_image_stats(env, cuda):
    """A narrow image (W = 16: one partial 64-pixel column tile per 6 rows) has
    more rows-kernel tiles than 128-pixel statistics slab rows; the launch
    caps its grid at the slab rows (each workgroup owns slab row blockIdx.x).
    Forward with dropout + BN sums (acfe_conv2d_fwd_dropout) against float64."""
    ops, call, lib, ptr, stream = env
    N, H, W, C, K = 2, 64, 16, 64, 64
    x, w, b, g = _data(N, H, W, C, K, 108, cuda)
    wp = ops.pack_weights(w, BF, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    # slab padded with sentinel rows: nothing may be written past `rows`
    st = torch.full((rows + 4, 2, wp.shape[0]), 7.0, dtype=F64, device=cuda)
    y0, y1 = (torch.empty((N, H, W, K), dtype=BF, device=cuda) for _ in range(2))
    call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y0), 1, None, stream())
    call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y1), 1,
         ptr(st), 0.1, 31, stream())
    torch.cuda.synchronize()
    _within_ulp(y0, _oracle_conv(x, w, b), what="narrow fwd")
    ref = torch.empty_like(y0)
    call("acfe_dropout", ptr(y0), y0.numel(), 0.1, 31, ptr(ref), 1, stream())
    torch.cuda.synchronize()
    assert torch.equal(y1, ref)
    torch.testing.assert_close(st[:rows].sum(0)[:, :K].cpu(), _sums(y1), rtol=1e-6, atol=1e-6)
    assert bool((st[rows:] == 7.0).all())


def test_head_conv_wgrad_row_halo(env, cuda):
    """wr_resnet_bird's head Conv2D (4, 10) 256 -> 128 at 16 x 32 (Keras
    "same": pad top 1 / bottom 2, left 4 / right 5; wr_resnet_bird.py:47-52):
    its weight gradient runs on k_wgrad_row_halo (one filter row x 64 channels
    x all 10 taps per workgroup, split-K + combine) -- at 32 clips, 16 per-row
    groups x the production split count -- against float64."""
    ops, call, lib, ptr, stream = env
    N, H, W, C, K, R, S = 32, 16, 32, 256, 128, 4, 10
    g = torch.Generator().manual_seed(11)
    x = (torch.randn((N, H, W, C), generator=g) * 0.5).to(BF).to(cuda)
    dy = (torch.randn((N, H, W, K), generator=g) * 0.5).to(BF).to(cuda)
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, R, S, H, W),), device=cuda)
    dw = torch.full((K, R, S, C), 7.0, device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, R, S, 1, 1, 4, H, W, ptr(dw), 0.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    xp = F.pad(x.cpu().to(F64).permute(0, 3, 1, 2), (4, 5, 1, 2))
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    dw_exact = torch.nn.grad.conv2d_weight(xp, (K, C, R, S), gd).permute(0, 2, 3, 1)
    d = dw.cpu().to(F64)
    assert ((d - dw_exact).norm() / dw_exact.norm()).item() < 5e-5
    assert ((d - dw_exact).abs().max() / dw_exact.abs().max()).item() < 5e-4
    # beta = 1 accumulates onto the previous gradient
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, R, S, 1, 1, 4, H, W, ptr(dw), 1.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    assert ((dw.cpu().to(F64) - 2 * dw_exact).norm() / (2 * dw_exact).norm()).item() < 5e-5


@pytest.mark.parametrize("C,K,H,W", [(128, 32, 32, 64), (256, 16, 16, 32), (64, 32, 20, 70), (32, 128, 32, 64),
                                     (32, 128, 13, 70), (32, 128, 16, 32), (16, 256, 16, 32), (16, 256, 13, 70)],
                         ids=["s2-128to32", "s3-256to16", "ragged", "c32-s2-32to128", "c32-ragged", "c32-narrow",
                              "c16-s3-16to256", "c16-256-ragged"])
def test_conv_narrow_production(env, cuda, C, K, H, W):
    """k_conv3x3_narrow (resident weights, halo staged once for all nine taps)
    at wr_resnet_bird's stage-2/3 branch21 shapes (128 -> 32 at 32 x 64,
    256 -> 16 at 16 x 32; 32 clips: more tiles than workgroups) and a ragged
    one (partial row and column tiles), and k_conv3x3_cw (32 -> 128 and
    16 -> 256: the stage-2 / 3 branch2b forwards and branch21 dgrads; 64- and
    32-pixel-wide tiles, ragged images): outputs within 1 bf16 ulp of the float64 conv, BN
    sums of the stored values to 1e-6, the fused Dropout's mask equal to
    acfe_dropout's, and the dgrad of the matching conv (dY K' = C channels ->
    dX K channels: 32 -> 128 / 16 -> 256 run on k_conv3x3_cw, 128 -> 32 and
    256 -> 16 on the narrow kernel)."""
    ops, call, lib, ptr, stream = env
    N = 32 if H * W <= 2048 else 8
    x, w, b, g = _data(N, H, W, C, K, 211 + K, cuda)
    wp = ops.pack_weights(w, BF, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    y = torch.empty((N, H, W, K), dtype=BF, device=cuda)
    st = torch.full((rows, 2, wp.shape[0]), 3.0, dtype=F64, device=cuda)
    call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y), 1, ptr(st),
         stream())
    yd = torch.empty_like(y)
    std = torch.empty_like(st)
    call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(yd), 1,
         ptr(std), 0.1, 977, stream())
    ref_drop = torch.empty_like(y)
    call("acfe_dropout", ptr(y), y.numel(), 0.1, 977, ptr(ref_drop), 1, stream())
    torch.cuda.synchronize()
    _within_ulp(y, _oracle_conv(x, w, b), what="narrow fwd")
    torch.testing.assert_close(st.sum(0)[:, :K].cpu(), _sums(y), rtol=1e-6, atol=1e-6)
    assert float(st[:, :, K:].abs().max()) == 0.0 if wp.shape[0] > K else True
    assert torch.equal(yd, ref_drop)
    torch.testing.assert_close(std.sum(0)[:, :K].cpu(), _sums(yd), rtol=1e-6, atol=1e-6)
    # dgrad of a K -> C... i.e. of the conv C' = K -> K' = C (branch2b): output K channels
    w2 = (torch.randn((C, 3, 3, K), generator=g) / (3 * K ** 0.5)).to(cuda)
    dy = (torch.randn((N, H, W, C), generator=g) * 0.5).to(BF).to(cuda)
    wf = ops.pack_weights(w2, BF, True)
    dx = torch.empty((N, H, W, K), dtype=BF, device=cuda)
    call("acfe_conv2d_dgrad", ptr(dy), N, H, W, C, ptr(wf), K, 3, 3, 1, 1, 1, H, W, ptr(dx), 1, None, stream())
    torch.cuda.synchronize()
    wd = w2.cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    gd = dy.cpu().to(F64).permute(0, 3, 1, 2)
    _within_ulp(dx, F.conv_transpose2d(gd, wd, padding=1).permute(0, 2, 3, 1), what="narrow dgrad")


@pytest.mark.parametrize("N,H,W,R,relu", [(3, 40, 130, 5, 0), (2, 37, 71, 3, 1), (2, 128, 513, 5, 0),
                                          (2, 33, 65, 5, 1)],
                         ids=["odd-5x5", "odd-3x3-relu", "t1-shape", "edge-5x5-relu"])
def test_stem_bwd_bn_fused(env, cuda, N, H, W, R, relu):
    """acfe_stem_bwd_bn (wr_resnet_bird.py:22-30: the stem conv's backward with
    its BN's backward apply folded into the dY staging) against the unfused
    chain acfe_bn_bwd_apply_ex -> acfe_stem_dgrad + acfe_stem_wgrad +
    acfe_channel_sum: dX bit-identical (same bf16 dX_bn and MFMA operands), dW
    within 1e-6 (the fused pass walks the tiles with fewer workgroups: another
    fp32 summation order) and the bias sums within 1e-6 of the sum of |dX_bn|
    (both add the same bf16 values in float64, in different orders)."""
    ops, call, lib, ptr, stream = env
    K, rep = 16, 3
    S = R
    pt = pl = (R - 1) // 2
    g = torch.Generator().manual_seed(29 + H + R)
    gy = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    xb = (torch.randn((N, H, W, K), generator=g) * 2).to(BF).to(cuda)
    xin = torch.randn((N, H, W), generator=g).to(BF).to(cuda)
    w = (torch.randn((K, R, S, rep), generator=g) * 0.2).to(cuda)
    sc = ((torch.rand(K, generator=g) + 0.5) * torch.where(torch.rand(K, generator=g) < 0.2, -1.0, 1.0)).to(cuda)
    sh = (torch.randn(K, generator=g) * 0.3).to(cuda)
    coef = (torch.randn(3 * K, generator=g) * 0.5).to(cuda)
    weff = torch.empty((R, S, K), device=cuda)
    call("acfe_stem_fold_weights", ptr(w), K, R, S, rep, ptr(weff), stream())
    rows = N * H * W
    nb = lib.acfe_stem_blocks(N, H, W)
    # unfused chain
    dxb = torch.empty((N, H, W, K), dtype=BF, device=cuda)
    call("acfe_bn_bwd_apply_ex", ptr(gy), 1, ptr(xb), 1, rows, K, ptr(sc), ptr(sh), relu, ptr(coef), None, 0.0, 0,
         ptr(dxb), 1, None, stream())
    dx0 = torch.empty((N, H, W), dtype=BF, device=cuda)
    call("acfe_stem_dgrad", ptr(dxb), 1, N, H, W, R, S, pt, pl, ptr(weff), ptr(dx0), 1, stream())
    dw0 = torch.empty((K, R, S, rep), device=cuda)
    ws0 = torch.empty((nb * K * R * S,), dtype=F64, device=cuda)
    call("acfe_stem_wgrad", ptr(xin), 1, ptr(dxb), 1, N, H, W, R, S, pt, pl, rep, ptr(dw0), 0.0, ptr(ws0), stream())
    db0 = torch.empty((K,), device=cuda)
    cpart = torch.empty((lib.acfe_reduce_blocks(rows) * 2 * K,), dtype=F64, device=cuda)
    call("acfe_channel_sum", ptr(dxb), rows, K, 1, ptr(cpart), ptr(db0), 0.0, stream())
    # fused
    dx1 = torch.full((N, H, W), float("nan"), dtype=BF, device=cuda)
    dw1 = torch.full((K, R, S, rep), float("nan"), device=cuda)
    ws1 = torch.empty((nb * K * R * S,), dtype=F64, device=cuda)
    bp = torch.full((nb, 2, K), float("nan"), dtype=F64, device=cuda)
    call("acfe_stem_bwd_bn", ptr(gy), ptr(xb), ptr(xin), N, H, W, R, S, pt, pl, ptr(weff), ptr(sc), ptr(sh),
         ptr(coef), relu, ptr(dx1), rep, ptr(dw1), 0.0, ptr(bp), ptr(ws1), stream())
    db1 = torch.empty((K,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(bp), nb, K, 0.0, ptr(db1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx1.view(torch.int16), dx0.view(torch.int16))
    assert ((dw1 - dw0).norm() / dw0.norm()).item() < 1e-6
    scale_ = dxb.float().abs().sum((0, 1, 2)).clamp_min(1.0)
    assert ((db1 - db0).abs() / scale_).max().item() < 1e-6
    ref = dxb.cpu().to(F64).sum((0, 1, 2))
    assert ((db1.cpu().to(F64) - ref).abs() / scale_.cpu().to(F64)).max().item() < 1e-6


def test_model_stem_bn_fusion(env, cuda):
    """A wr_resnet_bird training step with the stem node (acfe_stem_bwd_bn) on
    and off (ops.STEM_BN_FUSE): identical loss and every parameter gradient
    bit-identical except the stem conv's weight and bias (their sums are added
    in another order: within 1e-5)."""
    ops = env[0]
    from acfe.train import FrontEnd, Trainer
    from resnet.wr_resnet_bird import WRResNet
    import bench

    outs = []
    old = ops.STEM_BN_FUSE
    try:
        for f in (False, True):
            ops.STEM_BN_FUSE = f
            torch.manual_seed(0)
            model = WRResNet(input_shape=(128, 513, 3), classes=10, dtype=BF).to(cuda)
            fe = FrontEnd(n_mels=128, dtype=BF, device=cuda).to(cuda)
            tr = Trainer(model, fe, lr=0.0, loss="cce", device=cuda)
            x1, x2, lam, y = bench.make_batches(4, 10, cuda, n_sets=1)[0]
            ops._seed_counter = itertools.count()  # same dropout seeds in both runs
            loss, _ = tr.step(x1, y, x2, lam)
            torch.cuda.synchronize()
            names = [n for n, p in tr.holder.named_parameters() if p.requires_grad]
            outs.append((loss.detach().clone(), {n: tr.arena.grad[o:o + k].detach().clone()
                                                 for n, (o, k) in zip(names, tr.arena.offsets)}))
    finally:
        ops.STEM_BN_FUSE = old
    (l0, g0), (l1, g1) = outs
    assert torch.equal(l0, l1)
    assert any("conv1_1" in n for n in g0)
    for n in g0:
        if "conv1_1" in n:  # the stem weight and bias
            assert ((g1[n] - g0[n]).abs().max() / g0[n].abs().max().clamp_min(1e-30)).item() < 1e-5, n
        else:
            assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("C,K,H,W", [(128, 32, 32, 64), (32, 128, 32, 64), (32, 256, 16, 32), (16, 256, 16, 32),
                                     (64, 64, 64, 128), (128, 64, 64, 128), (64, 64, 14, 100), (256, 256, 22, 86),
                                     (256, 16, 16, 32), (128, 16, 16, 40), (16, 64, 64, 100), (16, 64, 15, 70),
                                     (64, 16, 20, 70), (128, 128, 22, 100), (64, 64, 10, 150)],
                         ids=["s2-21", "s2-2b", "s3-2b-b6", "s3-2b", "k64-rowpair", "k64-rowpair-2chunks",
                              "k64-rowpair-partial", "wrn-s3-256", "s3-21-k16", "k16-1chunk-partial",
                              "wrn-s1-2a-c16", "c16-k64-oddrows", "k16-c64-chunks", "k128-rem-oddrows",
                              "k64-rem-2cols"])
def test_wgrad_halo_narrow(env, cuda, C, K, H, W):
    """k_wgrad3x3_halo for the stage-2/3 layers whose channel count is the
    feature height: K = 32 (branch21 128 -> 32) and the 16 / 32-channel
    chunks (branch2b 32 -> 128 / 256, 16 -> 256), and the K = 64 layers'
    two-rows-per-step variant (k_wgrad3x3_halo<64, false, 64, 2>: 64 x 128
    stage-2 shapes, two 64-channel chunks, and a partial last column segment),
    and wr_resnet's stage-3 256 -> 256 at 22 x 86 (32-channel chunks of C),
    the K = 16 layers (128-channel chunks, one 16-channel block per wave; 64-
    channel chunks with two pixel groups when C = 64 * odd) and
    wr_resnet's stage-1 16 -> 64 (two pixel groups of waves writing separate
    split slabs; two rows per step, one for an odd row count), at 32 clips and
    the production split count, against float64.  Widths past a multiple of
    64 run their last Q % 64 pixels as 16-pixel segments (r06; a partial last
    row group at 22 / 10 rows, two remainder columns at W = 150)."""
    ops, call, lib, ptr, stream = env
    N = 32
    x, w, b, g = _data(N, H, W, C, K, 307, cuda)
    dy = (torch.randn((N, H, W, K), generator=g) * 0.5).to(BF).to(cuda)
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw = torch.empty((K, 3, 3, C), device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy), K, 3, 3, 1, 1, 1, H, W, ptr(dw), 0.0, 1, ptr(ws),
         stream())
    torch.cuda.synchronize()
    dw_exact = torch.nn.grad.conv2d_weight(x.cpu().to(F64).permute(0, 3, 1, 2), (K, C, 3, 3),
                                           dy.cpu().to(F64).permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    d = dw.cpu().to(F64)
    assert ((d - dw_exact).norm() / dw_exact.norm()).item() < 5e-5
    assert ((d - dw_exact).abs().max() / dw_exact.abs().max()).item() < 5e-4


def _bn_affine(C, seed, device):
    """scale / shift of a trained-looking BN (mixed signs so the ReLU cuts)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    sc = (torch.rand(C, generator=g) * 1.5 + 0.25) * torch.where(torch.rand(C, generator=g) < 0.1, -1.0, 1.0)
    sh = torch.randn(C, generator=g) * 0.5
    return sc.to(device), sh.to(device)


@pytest.mark.parametrize("N,H,W,C,K,mode", [(8, 64, 128, 64, 64, "drop"), (8, 64, 128, 128, 64, "add"),
                                            (4, 64, 128, 64, 64, "plain"), (3, 14, 100, 64, 64, "add"),
                                            (2, 9, 70, 128, 64, "drop"), (8, 64, 128, 64, 64, "pool"),
                                            (3, 14, 100, 64, 64, "pool"), (4, 64, 257, 128, 128, "drop"),
                                            (4, 64, 257, 128, 128, "add"), (2, 9, 70, 128, 128, "plain"),
                                            (3, 14, 100, 128, 128, "add")])
def test_conv_bn_prologue(env, cuda, N, H, W, C, K, mode):
    """acfe_conv2d_fwd_bn / acfe_conv2d_fwd_add_bn (BatchNormalization + ReLU
    applied while staging the conv input, resnet/wr_resnet_bird.py:136-161)
    against the unfused chain acfe_bn_apply -> acfe_conv2d_fwd_dropout /
    acfe_conv2d_fwd_add: the conv output, its BN statistics and the written BN
    output x' all bit-identical; x' also against the float64 BN of x within one
    bf16 ulp.  Shapes: the stage-1 layers (K = 64, C = 64 / 128) at production
    tile counts, plus partial 6-row / 64-column tiles; K = C = 128 (the
    one-wave kernel's prologue: wr_resnet's stage-2 bn2a / bn2b -> conv2a /
    conv2b at 64 x 257, a ragged image, no-dropout plain)."""
    ops, call, lib, ptr, stream = env
    assert lib.acfe_conv2d_bn_prologue_supported(N, H, W, C, K, 1)
    x, w, b, g = _data(N, H, W, C, K, 131 + C + H, cuda)
    sc, sh = _bn_affine(C, 7 + C, cuda)
    wp = ops.pack_weights(w, BF, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    res = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)

    def run(fused):
        xb = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
        if mode == "pool":
            y = torch.empty((N, H // 2, W // 2, K), dtype=BF, device=cuda)
            am = torch.empty((N, H // 2, W // 2, K), dtype=torch.uint8, device=cuda)
            st = torch.empty((rows, 2, wp.shape[0]), dtype=F64, device=cuda)
            if not fused:
                call("acfe_bn_apply", ptr(x), 1, N * H * W, C, ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
                call("acfe_conv2d_fwd_pool", ptr(xb), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(am), 0.1, 91,
                     ptr(st), 1, stream())
            else:
                call("acfe_conv2d_fwd_pool_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(am), 0.1,
                     91, ptr(st), ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
            torch.cuda.synchronize()
            return xb, torch.cat([y.view(torch.uint8).flatten(), am.flatten()]).view(torch.int16), st
        y = torch.empty((N, H, W, K), dtype=BF, device=cuda)
        st = torch.empty((rows, 2, wp.shape[0]), dtype=F64, device=cuda)
        if not fused:
            call("acfe_bn_apply", ptr(x), 1, N * H * W, C, ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
        if mode == "add":
            if fused:
                call("acfe_conv2d_fwd_add_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(res), 1, ptr(y),
                     ptr(st), ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
            else:
                call("acfe_conv2d_fwd_add", ptr(xb), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(res), 1, ptr(y),
                     ptr(st), 1, stream())
        else:
            rate = 0.1 if mode == "drop" else 0.0
            if fused:
                call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), rate, 77,
                     ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
            else:
                call("acfe_conv2d_fwd_dropout", ptr(xb), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b),
                     ptr(y), 1, ptr(st), rate, 77, stream())
        torch.cuda.synchronize()
        return xb, y, st

    xb0, y0, st0 = run(False)
    xb1, y1, st1 = run(True)
    assert torch.equal(xb1.view(torch.int16), xb0.view(torch.int16)), "BN output"
    assert torch.equal(y1.view(torch.int16), y0.view(torch.int16)), "conv output (+ argmax bytes)"
    assert torch.equal(st1[:, :, :K], st0[:, :, :K]), "BN statistics"
    exact = (x.cpu().to(F64) * sc.cpu().to(F64) + sh.cpu().to(F64)).clamp_min(0)
    _within_ulp(xb1, exact, atol=1e-6, what="x'")


def test_model_bn_prologue_matches_unfused(env, cuda):
    """A wr_resnet_bird training step with the BN prologue (the stage-1 BN ->
    ReLU -> conv pairs on acfe_conv2d_fwd_bn / fwd_add_bn) against the same
    step with every BN output written by its apply pass (ops.PROLOGUE off):
    identical loss, logits and gradients."""
    ops = env[0]
    from acfe.train import FrontEnd, Trainer
    from resnet.wr_resnet_bird import WRResNet
    import bench

    B = 4
    outs = []
    for pro in (False, True):
        ops.PROLOGUE = pro
        try:
            torch.manual_seed(0)
            model = WRResNet(input_shape=(128, 513, 3), classes=10, dtype=BF).to(cuda)
            fe = FrontEnd(n_mels=128, dtype=BF, device=cuda).to(cuda)
            tr = Trainer(model, fe, lr=0.01, loss="cce", device=cuda)
            x1, x2, lam, y = bench.make_batches(B, 10, cuda, n_sets=1)[0]
            ops._seed_counter = itertools.count()  # same dropout seeds in both runs
            loss, z = tr.step(x1, y, x2, lam)
            torch.cuda.synchronize()
            outs.append((loss.detach().clone(), tr.arena.grad.detach().clone(), tr.arena.flat.detach().clone()))
        finally:
            ops.PROLOGUE = True
    (l0, g0, p0), (l1, g1, p1) = outs
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("N,H,W,C,kh,kw,relu", [(8, 128, 513, 16, 1, 2, False), (4, 33, 70, 64, 2, 2, True),
                                                (2, 30, 45, 16, 3, 3, True)])
def test_maxpool_bwd_bn_reduce_fused(env, cuda, N, H, W, C, kh, kw, relu):
    """acfe_maxpool2d_bwd_argmax_bn (the stem BN -> MaxPool2D((1, 2)) backward,
    wr_resnet_bird.py:29-30, at the T1 shape; odd sizes whose edge rows /
    columns fall outside every window) against the unfused pair
    acfe_maxpool2d_bwd_argmax -> acfe_bn_bwd_reduce: the expanded gradient
    bit-identical, the reduce slab's per-channel column sums within 1e-9
    relative (both sum in fp32 partials and doubles, in different orders)."""
    ops, call, lib, ptr, stream = env
    g = torch.Generator().manual_seed(17 + H)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    sc = (torch.rand(C, generator=g) + 0.5).to(cuda)
    sh = (torch.randn(C, generator=g) * 0.3).to(cuda)
    mu = (torch.randn(C, generator=g) * 0.1).to(cuda)
    inv = (torch.rand(C, generator=g) + 0.5).to(cuda)
    P, Q = H // kh, W // kw
    y = torch.empty((N, P, Q, C), dtype=BF, device=cuda)
    am = torch.empty((N, P, Q, C), dtype=torch.uint8, device=cuda)
    call("acfe_bn_maxpool2d_fused", ptr(x), N, H, W, C, ptr(sc), ptr(sh), int(relu), kh, kw, ptr(y), ptr(am), None, 1,
         stream())
    dy = torch.randn((N, P, Q, C), generator=g).to(BF).to(cuda)
    rows = N * H * W
    nrows = lib.acfe_reduce_blocks(rows)
    gu0 = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    gu1 = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    part0 = torch.empty((nrows, 2, C), dtype=F64, device=cuda)
    part1 = torch.full((nrows, 2, C), float("nan"), dtype=F64, device=cuda)
    call("acfe_maxpool2d_bwd_argmax", ptr(am), ptr(dy), N, H, W, C, kh, kw, 0.0, 0, ptr(gu0), 1, stream())
    call("acfe_bn_bwd_reduce", ptr(gu0), 1, ptr(x), 1, rows, C, ptr(sc), ptr(sh), ptr(mu), ptr(inv), int(relu),
         ptr(part0), stream())
    call("acfe_maxpool2d_bwd_argmax_bn", ptr(am), ptr(dy), N, H, W, C, kh, kw, ptr(gu1), 1, ptr(x), ptr(sc), ptr(sh),
         ptr(mu), ptr(inv), int(relu), ptr(part1), stream())
    torch.cuda.synchronize()
    assert torch.equal(gu1.view(torch.int16), gu0.view(torch.int16))
    s0, s1 = part0.sum(0).cpu(), part1.sum(0).cpu()
    assert torch.isfinite(s1).all()
    # float64 reference of the sums
    gx = gu0.cpu().to(F64)
    xx = x.cpu().to(F64)
    if relu:
        gx = gx * ((xx * sc.cpu().to(torch.float32).to(F64) + sh.cpu().to(F64)) > 0)
    ref = torch.stack([gx.sum((0, 1, 2)), (gx * (xx - mu.cpu().to(F64)) * inv.cpu().to(F64)).sum((0, 1, 2))])
    scale_ = ref.abs().amax(1, keepdim=True).clamp_min(1.0)
    assert ((s1 - s0).abs() / scale_).max().item() < 1e-6, ((s1 - s0).abs() / scale_).max()
    assert ((s1 - ref).abs() / scale_).max().item() < 1e-5


@pytest.mark.parametrize("model_name", ["bird", "wrn"])
def test_model_bn_reduce_fusion_matches_unfused(env, cuda, model_name):
    """A training step with the BN backward reduces formed by the kernels that
    produce their gradients (ops.FUSE_BN_REDUCE: the stem BN's by the pool
    backward on wr_resnet_bird, bn2a / bn2b's by the 64-channel dgrads on
    wr_resnet) against the separate reduce passes: same loss and logits;
    gradients equal up to the sums' summation order."""
    ops = env[0]
    from acfe.train import FrontEnd, Trainer
    import bench

    B = 4
    outs = []
    old = ops.FUSE_BN_REDUCE
    for fuse in (False, True):
        ops.FUSE_BN_REDUCE = fuse
        try:
            torch.manual_seed(0)
            if model_name == "bird":
                from resnet.wr_resnet_bird import WRResNet
                model = WRResNet(input_shape=(128, 513, 3), classes=10, dtype=BF).to(cuda)
            else:
                from resnet.wr_resnet import WRResNet
                model = WRResNet(input_shape=(128, 513, 1), classes=10, dtype=BF).to(cuda)
            fe = FrontEnd(n_mels=128, dtype=BF, device=cuda).to(cuda)
            tr = Trainer(model, fe, lr=0.0, loss="cce", device=cuda)
            x1, x2, lam, y = bench.make_batches(B, 10, cuda, n_sets=1)[0]
            ops._seed_counter = itertools.count()  # same dropout seeds in both runs
            loss, z = tr.step(x1, y, x2, lam)
            torch.cuda.synchronize()
            names = [n for n, p in tr.holder.named_parameters() if p.requires_grad]
            outs.append((loss.detach().clone(), z.detach().clone(), tr.arena.grad.detach().clone()))
        finally:
            ops.FUSE_BN_REDUCE = old
    (l0, z0, g0), (l1, z1, g1) = outs
    assert torch.equal(l0, l1) and torch.equal(z0, z1)
    # Per parameter, in backward order (the arena is in registration order,
    # the head last): everything the backward computes before the first fused
    # BN is bit-identical, and the first parameter that differs is that BN's
    # gamma / beta gradient, off by the sums' summation order only (~1e-7) --
    # a wrong or dropped slab would show there at O(1).
    offs = tr.arena.offsets
    diff = [i for i, (o, k) in enumerate(offs) if not torch.equal(g0[o:o + k], g1[o:o + k])]
    assert diff, "the fused and unfused reduces gave bit-identical gradients: was the fusion exercised?"
    last = diff[-1]
    o, k = offs[last]
    first_rel = ((g1[o:o + k] - g0[o:o + k]).double().norm() / g0[o:o + k].double().norm()).item()
    assert "bn" in names[last] and first_rel < 1e-5, (names[last], first_rel)
    rel = ((g1.double() - g0.double()).norm() / g0.double().norm()).item()
    # The fused sums differ from the reduce pass's in summation order only
    # (~1e-7 relative: the first fused BN's gamma / beta gradients); each later
    # BN backward in bf16 turns that into rounding flips of its dX, and at
    # batch 4 the BN backwards amplify them ~3-10x per block towards the input
    # (per-parameter profiles, tools/dbg_bnfuse.py: bird r04j 1e-7 at
    # blocks.3.bn2b -> 5e-3 at the stem; wrn r04o 1e-7 at blocks.5.bn2b ->
    # 6e-3 at the stem, whole arena 3.2e-3), as they do any rounding
    # difference of the unfused chain.  The sums themselves: the op tests.
    # Bound: 3x the largest whole-arena difference measured (3.2e-3).
    assert rel < 1e-2, rel


@pytest.mark.parametrize("N,H,W,C,K,relu", [(4, 128, 513, 64, 64, True), (2, 21, 70, 64, 128, True),
                                              (3, 9, 64, 64, 64, False), (4, 64, 257, 128, 128, True),
                                              (3, 22, 100, 128, 128, False)])
def test_conv_dgrad_bn_reduce_fused(env, cuda, N, H, W, C, K, relu):
    """acfe_conv2d_dgrad_bn (wr_resnet's 64-channel bn2a / bn2b -> conv dgrads,
    resnet/wr_resnet.py:56-80, at the stage-1 128 x 513 shape; partial row /
    column tiles; no ReLU; and the stage-2 128 -> 128 dgrads at 64 x 257 on
    the one-wave kernel, r06) against acfe_conv2d_dgrad ->
    acfe_bn_bwd_reduce: dX bit-identical, the reduce slab's per-channel column
    sums within 1e-6 of each other and 1e-5 of a float64 sum (relative to the
    largest sum)."""
    ops, call, lib, ptr, stream = env
    g = torch.Generator().manual_seed(29 + W)
    dy = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    w = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    xb = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    sc = (torch.rand(C, generator=g) + 0.5).to(cuda)
    sh = (torch.randn(C, generator=g) * 0.3).to(cuda)
    mu = (torch.randn(C, generator=g) * 0.1).to(cuda)
    inv = (torch.rand(C, generator=g) + 0.5).to(cuda)
    wf = ops.pack_weights(w, BF, True)
    rows = N * H * W
    brows = lib.acfe_conv2d_dgrad_bn_rows(N, H, W, C, K, 3, 3, 1, 1)
    assert brows > 0
    assert lib.acfe_conv2d_dgrad_bn_rows(N, H, W, 32, K, 3, 3, 1, 1) == 0  # uncovered: C = 32
    assert lib.acfe_conv2d_dgrad_bn_rows(N, H, W, 128, 64, 3, 3, 1, 1) == 0  # uncovered: C = 128, K = 64
    dx0 = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    dx1 = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
    nrows = lib.acfe_reduce_blocks(rows)
    part0 = torch.empty((nrows, 2, C), dtype=F64, device=cuda)
    part1 = torch.full((brows, 2, C), float("nan"), dtype=F64, device=cuda)
    call("acfe_conv2d_dgrad", ptr(dy), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx0), 1, None, stream())
    call("acfe_bn_bwd_reduce", ptr(dx0), 1, ptr(xb), 1, rows, C, ptr(sc), ptr(sh), ptr(mu), ptr(inv), int(relu),
         ptr(part0), stream())
    call("acfe_conv2d_dgrad_bn", ptr(dy), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx1), 1, ptr(xb), ptr(sc),
         ptr(sh), ptr(mu), ptr(inv), int(relu), ptr(part1), brows, stream())
    torch.cuda.synchronize()
    assert torch.equal(dx1.view(torch.int16), dx0.view(torch.int16))
    s0, s1 = part0.sum(0).cpu(), part1.sum(0).cpu()
    assert torch.isfinite(s1).all()
    gx = dx0.cpu().to(F64)
    xx = xb.cpu().to(F64)
    if relu:
        gx = gx * ((xb.cpu().float() * sc.cpu() + sh.cpu()) > 0).to(F64)
    ref = torch.stack([gx.sum((0, 1, 2)), (gx * ((xb.cpu().float() - mu.cpu()) * inv.cpu()).to(F64)).sum((0, 1, 2))])
    scale_ = ref.abs().amax(1, keepdim=True).clamp_min(1.0)
    assert ((s1 - s0).abs() / scale_).max().item() < 1e-6, ((s1 - s0).abs() / scale_).max()
    assert ((s1 - ref).abs() / scale_).max().item() < 1e-5


@pytest.mark.parametrize("N,H,W,C,K,rate,relu", [(4, 128, 513, 64, 64, 0.1, 1), (8, 64, 128, 64, 64, 0.1, 1),
                                                 (2, 128, 513, 16, 64, 0.1, 1), (4, 32, 64, 128, 32, 0.1, 1),
                                                 (3, 14, 100, 64, 64, 0.0, 1), (2, 20, 70, 64, 64, 0.1, 0),
                                                 (2, 16, 64, 192, 64, 0.1, 1)],
                         ids=["wrn-s1-2a", "bird-s1-21", "wrn-s1b0-2a-c16", "bird-s2-21-k32", "partial-nodrop",
                              "norelu", "3chunks"])
def test_conv_wgrad_bnbwd_fused(env, cuda, N, H, W, C, K, rate, relu):
    """acfe_conv2d_wgrad_bnbwd (the BN backward apply of Conv2D -> Dropout ->
    BatchNormalization -> ReLU, resnet/wr_resnet.py:58-71 and
    resnet/wr_resnet_bird.py:139-154, formed while the halo wgrad stages its
    dY) against the unfused chain acfe_bn_bwd_apply_ex -> acfe_conv2d_wgrad +
    the apply pass's channel sums: the conv output gradient bit-identical, dW
    bit-identical (same staged values, same kernel and split), the bias sums
    within 1e-6 of the sum of |dy| (f32 partials of 16 segments vs per-element
    doubles).  Shapes: wr_resnet stage-1 (128 x 513, C = 64 and the C = 16
    block-0 conv2a), wr_resnet_bird stage 1 / stage-2 K = 32, a partial last
    column segment, no dropout, no ReLU, three chunks of C (only chunk 0's
    workgroups store and sum)."""
    ops, call, lib, ptr, stream = env
    srows = lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K)
    assert srows > 0
    g = torch.Generator().manual_seed(41 + H + C)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    gy = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    u = (torch.randn((N, H, W, K), generator=g) * 1.5).to(BF).to(cuda)
    sc = ((torch.rand(K, generator=g) + 0.5) * torch.where(torch.rand(K, generator=g) < 0.2, -1.0, 1.0)).to(cuda)
    sh = (torch.randn(K, generator=g) * 0.3).to(cuda)
    coef = (torch.randn(3 * K, generator=g) * 0.5).to(cuda)
    rows = N * H * W
    seed = 12345
    # unfused chain
    dy0 = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
    nr = lib.acfe_reduce_blocks(rows)
    sums0 = torch.empty((nr, 2, K), dtype=F64, device=cuda)
    call("acfe_bn_bwd_apply_ex", ptr(gy), 1, ptr(u), 1, rows, K, ptr(sc), ptr(sh), relu, ptr(coef), None, rate,
         seed, ptr(dy0), 1, ptr(sums0), stream())
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw0 = torch.empty((K, 3, 3, C), device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dy0), K, 3, 3, 1, 1, 1, H, W, ptr(dw0), 0.0, 1, ptr(ws),
         stream())
    db0 = torch.empty((K,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(sums0), nr, K, 0.0, ptr(db0), stream())
    # fused
    dy1 = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
    dw1 = torch.full((K, 3, 3, C), float("nan"), device=cuda)
    sums1 = torch.full((srows, 2, K), float("nan"), dtype=F64, device=cuda)
    ws1 = torch.empty_like(ws)
    call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(gy), ptr(u), K, ptr(sc), ptr(sh), relu, ptr(coef),
         None, rate, seed, ptr(dy1), ptr(dw1), 0.0, ptr(ws1), ptr(sums1), stream())
    db1 = torch.empty((K,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(sums1), srows, K, 0.0, ptr(db1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dy1.view(torch.int16), dy0.view(torch.int16)), "conv output gradient"
    assert torch.equal(dw1, dw0), ((dw1 - dw0).abs().max(), dw0.abs().max())
    scale_ = dy0.float().abs().sum((0, 1, 2)).clamp_min(1.0)
    assert ((db1 - db0).abs() / scale_).max().item() < 1e-6
    ref = dy0.cpu().to(F64).sum((0, 1, 2))
    assert ((db1.cpu().to(F64) - ref).abs() / scale_.cpu().to(F64)).max().item() < 1e-6
    # accumulate into an existing dW (beta 1, the arena path)
    dw2 = dw0.clone()
    call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(gy), ptr(u), K, ptr(sc), ptr(sh), relu, ptr(coef),
         None, rate, seed, ptr(dy1), ptr(dw2), 1.0, ptr(ws1), ptr(sums1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dw2, dw0 + dw0)


@pytest.mark.parametrize("model_name", ["bird", "wrn"])
def test_model_bn_bwd_fold_matches_unfused(env, cuda, model_name):
    """A training step with the Conv2D -> Dropout -> BN backward apply inside
    the wgrad (ops.FUSE_BN_BWD) against the separate apply pass: identical
    loss and logits, every parameter gradient bit-identical except the biases
    of the folded convs (their channel sums are added in another order: within
    1e-5 of max |grad|)."""
    ops = env[0]
    from acfe.train import FrontEnd, Trainer
    import bench

    outs = []
    old = ops.FUSE_BN_BWD
    try:
        for f in (False, True):
            ops.FUSE_BN_BWD = f
            torch.manual_seed(0)
            if model_name == "bird":
                from resnet.wr_resnet_bird import WRResNet
                model = WRResNet(input_shape=(128, 513, 3), classes=10, dtype=BF).to(cuda)
            else:
                from resnet.wr_resnet import WRResNet
                model = WRResNet(input_shape=(128, 513, 1), classes=10, dtype=BF).to(cuda)
            fe = FrontEnd(n_mels=128, dtype=BF, device=cuda).to(cuda)
            tr = Trainer(model, fe, lr=0.0, loss="cce", device=cuda)
            x1, x2, lam, y = bench.make_batches(4, 10, cuda, n_sets=1)[0]
            ops._seed_counter = itertools.count()  # same dropout seeds in both runs
            loss, z = tr.step(x1, y, x2, lam)
            torch.cuda.synchronize()
            names = [n for n, p in tr.holder.named_parameters() if p.requires_grad]
            outs.append((loss.detach().clone(), z.detach().clone(), tr.arena.grad.detach().clone()))
    finally:
        ops.FUSE_BN_BWD = old
    (l0, z0, g0), (l1, z1, g1) = outs
    assert torch.equal(l0, l1) and torch.equal(z0, z1)
    nbias = 0
    for n, (o, k) in zip(names, tr.arena.offsets):
        a, b = g0[o:o + k], g1[o:o + k]
        if torch.equal(a, b):
            continue
        # only conv biases may differ (summation order of the folded channel sums)
        assert n.endswith("bias") and "bn" not in n, n
        assert ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item() < 1e-5, n
        nbias += 1
    assert nbias > 0, "no conv bias differed: was the fold exercised?"


@pytest.mark.parametrize("N,H,W,C,K,mask_in", [(4, 128, 513, 64, 64, True), (8, 64, 128, 64, 64, False),
                                               (3, 14, 100, 64, 64, True)],
                         ids=["wrn-s1-2b", "bird-s1b0-2b-norelu", "partial"])
def test_conv_wgrad_bnbwd_residual(env, cuda, N, H, W, C, K, mask_in):
    """The residual form of acfe_conv2d_wgrad_bnbwd: conv2b's weight gradient
    forming the NEXT block's bn2a backward apply (resnet/wr_resnet.py:54-89:
    z = ReLU(conv2b + shortcut) is bn2a's input, the identity shortcut's
    gradient `add` is summed in, the ReLU of z masks the result) against
    acfe_bn_bwd_apply_ex(add, relu bit 1) -> acfe_conv2d_wgrad: dz
    bit-identical, dW bit-identical, bias sums within 1e-6."""
    ops, call, lib, ptr, stream = env
    srows = lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K)
    assert srows > 0
    g = torch.Generator().manual_seed(53 + H)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    gy = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    z = torch.randn((N, H, W, K), generator=g)
    z = (z.clamp_min(0) if mask_in else z).to(BF).to(cuda)
    add = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    sc = ((torch.rand(K, generator=g) + 0.5) * torch.where(torch.rand(K, generator=g) < 0.2, -1.0, 1.0)).to(cuda)
    sh = (torch.randn(K, generator=g) * 0.3).to(cuda)
    coef = (torch.randn(3 * K, generator=g) * 0.5).to(cuda)
    flags = 1 | (2 if mask_in else 0)
    rows = N * H * W
    dz0 = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
    nr = lib.acfe_reduce_blocks(rows)
    sums0 = torch.empty((nr, 2, K), dtype=F64, device=cuda)
    call("acfe_bn_bwd_apply_ex", ptr(gy), 1, ptr(z), 1, rows, K, ptr(sc), ptr(sh), flags, ptr(coef), ptr(add), 0.0,
         0, ptr(dz0), 1, ptr(sums0), stream())
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw0 = torch.empty((K, 3, 3, C), device=cuda)
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dz0), K, 3, 3, 1, 1, 1, H, W, ptr(dw0), 0.0, 1, ptr(ws),
         stream())
    db0 = torch.empty((K,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(sums0), nr, K, 0.0, ptr(db0), stream())
    dz1 = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
    dw1 = torch.full((K, 3, 3, C), float("nan"), device=cuda)
    sums1 = torch.full((srows, 2, K), float("nan"), dtype=F64, device=cuda)
    call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(gy), ptr(z), K, ptr(sc), ptr(sh), flags, ptr(coef),
         ptr(add), 0.0, 0, ptr(dz1), ptr(dw1), 0.0, ptr(ws), ptr(sums1), stream())
    db1 = torch.empty((K,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(sums1), srows, K, 0.0, ptr(db1), stream())
    torch.cuda.synchronize()
    assert torch.equal(dz1.view(torch.int16), dz0.view(torch.int16)), "dz"
    assert torch.equal(dw1, dw0)
    scale_ = dz0.float().abs().sum((0, 1, 2)).clamp_min(1.0)
    assert ((db1 - db0).abs() / scale_).max().item() < 1e-6
