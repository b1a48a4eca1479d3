"""GPU parity of the model kernels (HIP via the C ABI) against torch-CPU float64.

Tolerances:
  fp32 path (exact-fp32 MFMA 16x16x4): rel-L2 <= 1e-5 (fwd), 1e-5 (dgrad/wgrad)
  bf16 path: inputs/weights rounded to bf16 on both sides, fp32 accumulation,
             bf16 output rounding -> rel-L2 <= 6e-3 (fwd), 1e-2 (grads)
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from oracle.models import avgpool_same, conv as ref_conv, logmeanexp as ref_lme  # noqa: E402


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def rnd(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float64) * scale


@pytest.fixture(scope="module")
def ops(cuda):
    from acfe import ops as o

    return o


CONV_CASES = [
    # N, H, W, C, K, R, S, stride, padding
    (2, 16, 24, 16, 128, 1, 1, 1, "same"),
    (2, 16, 20, 128, 128, 3, 3, 1, "same"),
    (2, 12, 20, 64, 64, 3, 3, 1, "same"),
    (2, 9, 13, 32, 256, 3, 3, 1, "same"),
    (2, 8, 16, 256, 16, 3, 3, 1, "same"),
    (2, 16, 32, 256, 128, 4, 10, 1, "same"),
    (2, 16, 32, 256, 50, 1, 1, 1, "same"),
    (2, 16, 32, 50, 64, 3, 3, 1, "same"),
    (2, 7, 9, 4, 32, 3, 3, 1, "same"),
    (2, 16, 33, 64, 128, 3, 3, 2, "same"),
    (2, 16, 33, 64, 128, 1, 1, 2, "valid"),
    (2, 22, 31, 128, 256, 3, 3, 3, "same"),
    (2, 22, 31, 128, 256, 1, 1, 3, "valid"),
    # strided dgrad by sub-pixel phases: even sizes (pad_top 0), "valid" 3x3,
    # stride 3 with every phase offset, a phase with more taps than rows
    (2, 16, 34, 64, 128, 3, 3, 2, "same"),
    (2, 21, 29, 64, 64, 3, 3, 2, "valid"),
    (2, 23, 35, 64, 128, 3, 3, 3, "same"),
    (2, 3, 5, 64, 64, 3, 3, 2, "same"),
    (1, 300, 5, 16, 64, 3, 3, 1, "same"),
    # 16 input channels, 64 outputs (k_conv3x3_c16): ragged row / column tiles
    (2, 20, 70, 16, 64, 3, 3, 1, "same"),
    # halo-staged 3x3 wgrad (Q % 64 == 0, C % 64 == 0, K in {64, 128}): 1-3 channel chunks
    (2, 10, 64, 128, 128, 3, 3, 1, "same"),
    (2, 9, 128, 64, 64, 3, 3, 1, "same"),
    (1, 6, 64, 192, 128, 3, 3, 1, "same"),
    # r05 sweep of the dispatch paths at ragged sizes: rows K = 64 / one-wave
    # K = 128 with partial row and column tiles, c16, narrow K = 32 / 16, cw
    # (32 -> 128, 16 -> 256), a stride-2 "valid" 3x3 and 1x1 at odd sizes,
    # a K = 192 generic layer
    (2, 13, 70, 64, 64, 3, 3, 1, "same"),
    (1, 9, 130, 128, 128, 3, 3, 1, "same"),
    (2, 7, 33, 16, 64, 3, 3, 1, "same"),
    (2, 10, 20, 128, 32, 3, 3, 1, "same"),
    (2, 12, 24, 256, 16, 3, 3, 1, "same"),
    (2, 12, 24, 32, 128, 3, 3, 1, "same"),
    (2, 6, 40, 16, 256, 3, 3, 1, "same"),
    (1, 5, 7, 64, 64, 3, 3, 2, "valid"),
    (2, 11, 13, 64, 128, 1, 1, 2, "valid"),
    (2, 9, 17, 64, 192, 3, 3, 1, "same"),
    # register-weight 1x1 kernel (C or K <= 32)
    (2, 18, 30, 16, 64, 1, 1, 1, "valid"),
    (2, 11, 37, 32, 96, 1, 1, 1, "same"),
    (2, 11, 37, 128, 32, 1, 1, 1, "same"),
]


def _keras_out(n, k, s, padding):
    return -(-n // s) if padding == "same" else (n - k) // s + 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: "x".join(map(str, c[:8])) + c[8])
def test_conv_fwd_dgrad_wgrad(ops, cuda, case, dtype):
    N, H, W, C, K, R, S, st, pad = case
    x = rnd((N, H, W, C), 1)
    w = rnd((K, R, S, C), 2, 1.0 / math.sqrt(R * S * C))
    b = rnd((K,), 3, 0.1)
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).double()
        wq = w.to(torch.bfloat16).double()
    else:
        wq = w
    P, Q = _keras_out(H, R, st, pad), _keras_out(W, S, st, pad)
    gy = rnd((N, P, Q, K), 4)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).double()
    # reference (float64, NCHW)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wr = wq.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = ref_conv(xr, wr, br, st, pad)
    (yr * gy.permute(0, 3, 1, 2)).sum().backward()
    # device
    xd = x.to(dtype).to(cuda).requires_grad_(True)
    wd = w.float().to(cuda).requires_grad_(True)
    bd = b.float().to(cuda).requires_grad_(True)
    yd, _ = ops.conv2d(xd, wd, bd, st, pad)
    assert yd.shape == (N, P, Q, K)
    yd.backward(gy.to(dtype).to(cuda))
    tol = 1e-5 if dtype == torch.float32 else 6e-3
    assert rel(yd.float(), yr.permute(0, 2, 3, 1)) < tol
    gt = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(xd.grad.float(), xr.grad.permute(0, 2, 3, 1)) < gt
    assert rel(wd.grad, wr.grad) < gt
    assert rel(bd.grad, br.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


# bf16 shapes large enough that the persistent 3-stage kernel (k_conv_fwd_p:
# 256-row tiles, one workgroup per CU) walks several M tiles per workgroup,
# with a ragged last tile, nkt = 1 / 2 / 9 / 18 K-tiles, and two N tiles.
BIG_CASES = [
    (2, 128, 512, 64, 64, 3, 3),
    (1, 128, 515, 128, 128, 3, 3),
    (2, 128, 300, 16, 128, 1, 1),
    (1, 128, 600, 128, 64, 1, 1),
    (1, 64, 520, 128, 256, 3, 3),
    (2, 128, 513, 16, 64, 3, 3),  # wr_resnet's 16 -> 64 conv at the T1 input (k_conv3x3_c16, many tiles per CU)
]


@pytest.mark.parametrize("case", BIG_CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_pipelined_multi_tile(ops, cuda, case):
    N, H, W, C, K, R, S = case
    x = rnd((N, H, W, C), 11).to(torch.bfloat16).double()
    w = rnd((K, R, S, C), 12, 1.0 / math.sqrt(R * S * C))
    wq = w.to(torch.bfloat16).double()
    b = rnd((K,), 13, 0.1)
    gy = rnd((N, H, W, K), 14).to(torch.bfloat16).double()
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wr = wq.clone().requires_grad_(True)
    yr = ref_conv(xr, wr, b, 1, "same")
    (yr * gy.permute(0, 3, 1, 2)).sum().backward()
    xd = x.to(torch.bfloat16).to(cuda).requires_grad_(True)
    wd = w.float().to(cuda).requires_grad_(True)
    yd, st = ops.conv2d(xd, wd, b.float().to(cuda), 1, "same", want_stats=True)
    yd.backward(gy.to(torch.bfloat16).to(cuda))
    assert rel(yd.float(), yr.permute(0, 2, 3, 1)) < 6e-3
    assert rel(xd.grad.float(), xr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert rel(wd.grad, wr.grad) < 1e-2
    # BN partial statistics of the rounded outputs (every stats row written)
    yf = yd.detach().float().cpu().double()
    s = st.cpu().sum(0)
    np.testing.assert_allclose(s[0, :K].numpy(), yf.sum((0, 1, 2)).numpy(), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[1, :K].numpy(), (yf ** 2).sum((0, 1, 2)).numpy(), rtol=1e-5, atol=1e-3)


def test_conv_fused_bn_stats(ops, cuda):
    x = rnd((2, 10, 12, 64), 5).to(torch.bfloat16)
    w = rnd((64, 3, 3, 64), 6, 1 / 24)
    y, st = ops.conv2d(x.to(cuda), w.float().to(cuda), torch.zeros(64, device=cuda), 1, "same", want_stats=True)
    yf = y.float().cpu().double()
    s = st.cpu().sum(0)
    # per-tile partials are accumulated in fp32 before the double merge
    np.testing.assert_allclose(s[0, :64].numpy(), yf.sum((0, 1, 2)).numpy(), rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(s[1, :64].numpy(), (yf ** 2).sum((0, 1, 2)).numpy(), rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("R", [5, 3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_stem_folded(ops, cuda, R, dtype):
    N, H, W = 2, 20, 70
    m = rnd((N, H, W), 7)
    if dtype == torch.bfloat16:
        m = m.to(torch.bfloat16).double()
    w = rnd((16, R, R, 3), 8, 0.2)
    b = rnd((16,), 9, 0.1)
    xr = m[:, None].repeat(1, 3, 1, 1).requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = ref_conv(xr, wr, br)
    gy = rnd((N, H, W, 16), 10)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).double()
    (yr * gy.permute(0, 3, 1, 2)).sum().backward()
    xd = m.to(dtype).to(cuda).requires_grad_(True)
    wd, bd = w.float().to(cuda).requires_grad_(True), b.float().to(cuda).requires_grad_(True)
    yd, st = ops.stem_conv(xd, wd, bd, dtype, want_stats=True)
    yd.backward(gy.to(dtype).to(cuda))
    tol = 1e-5 if dtype == torch.float32 else 6e-3
    assert rel(yd.float(), yr.permute(0, 2, 3, 1)) < tol
    # d input of the folded map = sum over the 3 channel copies
    assert rel(xd.grad.float(), xr.grad.sum(1)) < (1e-5 if dtype == torch.float32 else 1e-2)
    assert rel(wd.grad, wr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    assert rel(bd.grad, br.grad) < 1e-5
    ys = yd.detach().float().cpu().double()
    np.testing.assert_allclose(st.cpu().sum(0)[0].numpy(), ys.sum((0, 1, 2)).numpy(), rtol=1e-9, atol=1e-6)


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_batchnorm_train(ops, cuda, relu, dtype):
    x = rnd((4, 6, 7, 48), 11, 2.0) + 0.5
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).double()
    g, b = rnd((48,), 12, 0.3) + 1, rnd((48,), 13, 0.3)
    gy = rnd(x.shape, 14)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).double()
    xr, gr, br = x.clone().requires_grad_(True), g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    mean, var = xr.mean((0, 1, 2)), xr.var((0, 1, 2), unbiased=False)
    yr = (xr - mean) / torch.sqrt(var + 1e-3) * gr + br
    if relu:
        yr = torch.relu(yr)
    (yr * gy).sum().backward()
    mm, mv = torch.zeros(48, device=cuda), torch.ones(48, device=cuda)
    xd = x.to(dtype).to(cuda).requires_grad_(True)
    gd, bd = g.float().to(cuda).requires_grad_(True), b.float().to(cuda).requires_grad_(True)
    yd = ops.batch_norm(xd, gd, bd, mm, mv, True, relu)
    yd.backward(gy.to(dtype).to(cuda))
    tol = 1e-5 if dtype == torch.float32 else 6e-3
    assert rel(yd.float(), yr) < tol
    gt = 1e-4 if dtype == torch.float32 else 1e-2
    assert rel(xd.grad.float(), xr.grad) < gt
    assert rel(gd.grad, gr.grad) < gt and rel(bd.grad, br.grad) < gt
    np.testing.assert_allclose(mm.cpu().numpy(), (0.01 * mean).detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(mv.cpu().numpy(), (0.99 + 0.01 * var).detach().numpy(), rtol=1e-5)
    # eval mode uses the moving statistics
    ye = ops.batch_norm(x.to(dtype).to(cuda), gd.detach(), bd.detach(), mm, mv, False, relu)
    ref_e = (x - mm.cpu().double()) / torch.sqrt(mv.cpu().double() + 1e-3) * g + b
    if relu:
        ref_e = torch.relu(ref_e)
    assert rel(ye.float(), ref_e) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_pools_dropout_add(ops, cuda, dtype):
    x = rnd((2, 8, 13, 16), 15)
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).double()
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, (2, 2), (2, 2))
    g = rnd(yr.shape, 16)
    (yr * g).sum().backward()
    xd = x.to(dtype).to(cuda).requires_grad_(True)
    yd = ops.max_pool(xd, 2, 2)
    yd.backward(g.permute(0, 2, 3, 1).to(dtype).to(cuda))
    assert torch.equal(yd.float().cpu(), yr.permute(0, 2, 3, 1).float())
    assert rel(xd.grad.float(), xr.grad.permute(0, 2, 3, 1)) < 1e-2
    # avg pool "same" with an odd width
    xr2 = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr2 = avgpool_same(xr2, 2)
    g2 = rnd(yr2.shape, 17)
    (yr2 * g2).sum().backward()
    xd2 = x.to(dtype).to(cuda).requires_grad_(True)
    yd2 = ops.avg_pool_same(xd2, 2)
    yd2.backward(g2.permute(0, 2, 3, 1).to(dtype).to(cuda))
    tol = 1e-6 if dtype == torch.float32 else 6e-3
    assert rel(yd2.float(), yr2.permute(0, 2, 3, 1)) < tol
    assert rel(xd2.grad.float(), xr2.grad.permute(0, 2, 3, 1)) < max(tol, 6e-3 if dtype == torch.bfloat16 else 0)
    # dropout: keep-rate and scaling, mask regenerated in backward
    ones = torch.ones((1 << 20,), device=cuda, dtype=dtype, requires_grad=True)
    yd3 = ops.dropout(ones, 0.1, True, seed=1234)
    kept = (yd3.float() != 0).float().mean().item()
    assert abs(kept - 0.9) < 3e-3
    assert torch.allclose(yd3.float()[yd3.float() != 0], torch.tensor(1 / 0.9, device=cuda), rtol=8e-3)
    yd3.backward(torch.ones_like(yd3))
    assert torch.equal(ones.grad.float() != 0, yd3.float() != 0)
    # add (+relu)
    a, b = rnd((1000,), 18).to(dtype).to(cuda), rnd((1000,), 19).to(dtype).to(cuda)
    z = ops.add(a, b, relu=True)
    assert rel(z.float(), torch.relu(a.double().cpu() + b.double().cpu())) < (1e-7 if dtype == torch.float32 else 5e-3)


@pytest.mark.parametrize("B,I,O", [(512, 32, 50), (70, 17, 3), (1, 5, 2)])
def test_dense_backward_batch_sizes(ops, cuda, B, I, O):
    """acfe_dense_bwd's weight / bias gradients (one wave per output striding
    the batch, float64 butterfly) against float64 autograd, at the T1 head's
    [512, 32] x [32, 50] and ragged batches."""
    x, w, b = rnd((B, I), 41), rnd((I, O), 42, 0.5), rnd((O,), 43, 0.1)
    dz = rnd((B, O), 44)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    (xr @ wr + br).backward(dz)
    xd, wd, bd = (t.float().to(cuda).requires_grad_(True) for t in (x, w, b))
    ops.dense(xd, wd, bd).backward(dz.float().to(cuda))
    assert rel(wd.grad, wr.grad) < 1e-6 and rel(bd.grad, br.grad) < 1e-6 and rel(xd.grad, xr.grad) < 1e-6


def test_lme_large_and_nonfinite(ops, cuda):
    """logmeanexp at the magnitudes an eval forward reaches with the Keras
    moving statistics still near their initial values (|x| ~ 1e9, found as a
    run-to-run NaN in test_train_checkpoint_predict[raw]: a contracted
    fma(s, x, -max) kept the max element's rounding residual in the exponent,
    expf(~256) = inf), and tfp.math.reduce_logsumexp's handling of an infinite
    max (shift by 0: +inf stays +inf, an all -inf row gives -inf, no NaN)."""
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((4, 16, 7, 3), generator=g, dtype=torch.float64) * 2 - 1) * 1.2e9
    x = x.float().double()  # the fp32 values the kernel sees
    ref = ref_lme(x, 1)
    y = ops.logmeanexp(x.float().to(cuda), 1).double().cpu()
    assert torch.isfinite(y).all()
    assert ((y - ref).abs() <= 1e-6 * ref.abs() + 1.0).all()
    xg = x.float().to(cuda).requires_grad_(True)
    ops.logmeanexp(xg, 1).sum().backward()
    xr = x.clone().requires_grad_(True)
    ref_lme(xr, 1).sum().backward()
    assert torch.isfinite(xg.grad).all() and (xg.grad.double().cpu() - xr.grad).abs().max() < 1e-5
    z = torch.tensor([[1.0, float("inf"), -2.0], [float("-inf")] * 3, [float("inf"), float("-inf"), 0.0]])
    yz = ops.logmeanexp(z.to(cuda), 1).cpu()
    assert yz[0] == float("inf") and yz[1] == float("-inf") and yz[2] == float("inf"), yz


def test_lme_dense_loss_adam(ops, cuda):
    from oracle.models import keras_adam, keras_loss

    x = rnd((3, 4, 6, 5), 20)
    xr = x.clone().requires_grad_(True)
    yr = ref_lme(ref_lme(xr, 1), 2)  # [3, 6]
    w, b = rnd((6, 5), 21, 0.5), rnd((5,), 22, 0.1)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    zr = yr @ wr + br
    tgt = torch.zeros(3, 5, dtype=torch.float64)
    tgt[0, 1] = tgt[1, 3] = tgt[2, 0] = 1
    for mode in ("cce", "bce"):
        for t in (xr, wr, br):
            t.grad = None
        lr_ = keras_loss(zr, tgt, mode)
        lr_.backward(retain_graph=True)
        xd = x.float().to(cuda).requires_grad_(True)
        wd, bd = w.float().to(cuda).requires_grad_(True), b.float().to(cuda).requires_grad_(True)
        yd = ops.logmeanexp(ops.logmeanexp(xd, 1), 2)
        zd = ops.dense(yd, wd, bd)
        ld, dz = ops.loss_and_grad(zd, tgt.float().to(cuda), mode)
        zd.backward(dz)
        assert abs(ld.item() - lr_.item()) < 1e-5 * max(1, abs(lr_.item()))
        assert rel(zd, zr) < 1e-6
        assert rel(xd.grad, xr.grad) < 1e-5 and rel(wd.grad, wr.grad) < 1e-5 and rel(bd.grad, br.grad) < 1e-5
    # Adam (Keras formulation), two steps
    from acfe.layers import Adam, ParamArena

    mod = torch.nn.Linear(4, 3).to(cuda)
    arena = ParamArena(mod, cuda)
    opt = Adam(arena, lr=0.01)
    params = [p.detach().double().cpu().clone() for p in arena.params]
    m = [torch.zeros_like(p) for p in params]
    v = [torch.zeros_like(p) for p in params]
    for t in (1, 2):
        grads = [rnd(p.shape, 30 + t + i) for i, p in enumerate(params)]
        arena.zero_grad()
        for p, g in zip(arena.params, grads):
            p.grad.copy_(g.float())
        opt.step()
        params, m, v = keras_adam(params, grads, m, v, t)
    for p, r in zip(arena.params, params):
        assert rel(p, r) < 1e-6
