"""GPU parity of the fused nodes against the same kernels run one op at a time.

Kernel level (bit-exact: the fused kernels must store exactly what the
separate kernels store):
  acfe_conv2d_fwd_dropout      == acfe_conv2d_fwd -> acfe_dropout
  acfe_bn_bwd_apply_dropout    == acfe_bn_bwd_apply -> acfe_dropout
  acfe_maxpool2d_fused         == acfe_maxpool2d -> acfe_dropout (+ argmax bytes)
  acfe_maxpool2d_bwd_argmax    == acfe_dropout -> acfe_maxpool2d_bwd
  acfe_add_stats               == acfe_add
Statistics slabs (different partial grouping) agree to rel 1e-6 with
acfe_bn_stats of the stored tensor.
Node level (autograd): conv_dropout_bn / maxpool_dropout_bn / the
ResidualLink'd block against the unfused op chain, rel-L2 <= 2e-3 on bf16
outputs and gradients (BN statistics summed in a different order can move a
bf16 rounding by one ulp).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def env(cuda):
    from acfe import ops
    from acfe._lib import call, lib
    from acfe._torch import ptr, stream

    return ops, call, lib, ptr, stream


def _stats_of(env, t):
    ops, call, lib, ptr, stream = env
    C = t.shape[-1]
    rows = t.numel() // C
    part = torch.empty((lib.acfe_reduce_blocks(rows), 2, C), dtype=torch.float64, device=t.device)
    call("acfe_bn_stats", ptr(t), rows, C, 1 if t.dtype == torch.bfloat16 else 0, ptr(part), stream())
    return part.sum(0)


def _dropout(env, t, rate, seed):
    ops, call, lib, ptr, stream = env
    y = torch.empty_like(t)
    call("acfe_dropout", ptr(t), t.numel(), rate, seed, ptr(y), 1 if t.dtype == torch.bfloat16 else 0, stream())
    return y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
@pytest.mark.parametrize("K,C", [(128, 64), (64, 64), (32, 64), (64, 16), (128, 128)],
                         ids=["128", "64", "32", "64c16", "128c128"])
def test_conv_fwd_dropout(env, cuda, dtype, K, C):
    """(C = 16, K = 64 bf16: k_conv3x3_c16, the tap-major 16-channel kernel;
    K = C = 128 bf16: the one-wave k_conv3x3_1w<0> with the dropout and BN sums
    between the next tile's MFMA groups, H = 12: a partial last row tile)"""
    ops, call, lib, ptr, stream = env
    N, H, W, R = 2, 12, 40, 3
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn((N, H, W, C), generator=g).to(dtype).to(cuda)
    w = (torch.randn((K, R, R, C), generator=g) * 0.05).to(cuda)
    b = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    dt = 1 if dtype == torch.bfloat16 else 0
    wp = ops.pack_weights(w, dtype, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    y0 = torch.empty((N, H, W, K), dtype=dtype, device=cuda)
    y1 = torch.empty_like(y0)
    st = torch.zeros((rows, 2, wp.shape[0]), dtype=torch.float64, device=cuda)
    call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, R, R, 1, 1, 1, H, W, ptr(b), ptr(y0), dt, None, stream())
    call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, R, R, 1, 1, 1, H, W, ptr(b), ptr(y1), dt,
         ptr(st), 0.1, 12345, stream())
    ref = _dropout(env, y0, 0.1, 12345)
    assert torch.equal(y1, ref)
    assert (ref == 0).float().mean().item() == pytest.approx(0.1, abs=0.02)
    s_ref = _stats_of(env, ref)
    # the epilogue sums each wave's 16-row fragment in fp32 before the double atomics
    torch.testing.assert_close(st.sum(0)[:, :K], s_ref, rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize("relu", [False, True])
def test_bn_bwd_apply_dropout(env, cuda, relu):
    ops, call, lib, ptr, stream = env
    rows, C = 3000, 64
    g = torch.Generator(device="cpu").manual_seed(2)
    dy = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    x = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    scale, shift, coef = (torch.randn((n,), generator=g).to(cuda) for n in (C, C, 3 * C))
    d0 = torch.empty_like(x)
    d1 = torch.empty_like(x)
    call("acfe_bn_bwd_apply", ptr(dy), 1, ptr(x), 1, rows, C, ptr(scale), ptr(shift), int(relu), ptr(coef), None,
         ptr(d0), 1, stream())
    call("acfe_bn_bwd_apply_dropout", ptr(dy), 1, ptr(x), 1, rows, C, ptr(scale), ptr(shift), int(relu), ptr(coef),
         0.1, 777, ptr(d1), 1, stream())
    assert torch.equal(d1, _dropout(env, d0, 0.1, 777))


@pytest.mark.parametrize("k", [(1, 2), (2, 2), (3, 3)])
@pytest.mark.parametrize("C", [16, 64, 128])
def test_maxpool_fused(env, cuda, k, C):
    ops, call, lib, ptr, stream = env
    kh, kw = k
    N, H, W = 2, 13, 35
    P, Q = H // kh, W // kw
    g = torch.Generator(device="cpu").manual_seed(3)
    # coarse values so ties occur (first maximum must win in both paths)
    x = (torch.randint(-4, 5, (N, H, W, C), generator=g).float() * 0.5).to(torch.bfloat16).to(cuda)
    y0 = torch.empty((N, P, Q, C), dtype=torch.bfloat16, device=cuda)
    call("acfe_maxpool2d", ptr(x), N, H, W, C, kh, kw, ptr(y0), 1, stream())
    ref = _dropout(env, y0, 0.1, 99)
    y1 = torch.empty_like(y0)
    am = torch.empty((N, P, Q, C), dtype=torch.uint8, device=cuda)
    st = torch.empty((lib.acfe_reduce_blocks(N * P * Q), 2, C), dtype=torch.float64, device=cuda)
    call("acfe_maxpool2d_fused", ptr(x), N, H, W, C, kh, kw, ptr(y1), ptr(am), 0.1, 99, ptr(st), 1, stream())
    assert torch.equal(y1, ref)
    torch.testing.assert_close(st.sum(0), _stats_of(env, ref), rtol=1e-6, atol=1e-6)
    # backward from the argmax bytes == dropout backward then maxpool backward from x
    gy = torch.randn((N, P, Q, C), generator=g).to(torch.bfloat16).to(cuda)
    dx0 = torch.empty_like(x)
    call("acfe_maxpool2d_bwd", ptr(x), ptr(_dropout(env, gy, 0.1, 99)), N, H, W, C, kh, kw, ptr(dx0), 1, stream())
    dx1 = torch.full_like(x, 7.0)  # leftover rows/cols must be overwritten with zeros
    call("acfe_maxpool2d_bwd_argmax", ptr(am), ptr(gy), N, H, W, C, kh, kw, 0.1, 99, ptr(dx1), 1, stream())
    assert torch.equal(dx1, dx0)


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("C", [16, 64, 256])
def test_add_stats(env, cuda, relu, C):
    ops, call, lib, ptr, stream = env
    rows = 5000
    g = torch.Generator(device="cpu").manual_seed(4)
    a = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    b = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    z0, z1 = torch.empty_like(a), torch.empty_like(a)
    call("acfe_add", ptr(a), ptr(b), a.numel(), int(relu), ptr(z0), 1, stream())
    st = torch.empty((lib.acfe_reduce_blocks(rows), 2, C), dtype=torch.float64, device=cuda)
    call("acfe_add_stats", ptr(a), ptr(b), rows, C, int(relu), ptr(z1), 1, ptr(st), stream())
    assert torch.equal(z1, z0)
    torch.testing.assert_close(st.sum(0), _stats_of(env, z0), rtol=1e-6, atol=1e-6)


def _bn_params(C, cuda, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    gamma = (1 + 0.2 * torch.randn((C,), generator=g)).to(cuda).requires_grad_(True)
    beta = (0.1 * torch.randn((C,), generator=g)).to(cuda).requires_grad_(True)
    return gamma, beta, torch.zeros(C, device=cuda), torch.ones(C, device=cuda)


@pytest.mark.parametrize("stride", [1, 2])
def test_conv_dropout_bn_node(env, cuda, stride):
    ops = env[0]
    N, H, W, C, K = 4, 16, 24, 32, 64
    g = torch.Generator(device="cpu").manual_seed(5)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 3, 3, C), generator=g) * 0.1).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gy = torch.randn((N, -(-H // stride), -(-W // stride), K), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(K, cuda, 6)
        if fused:
            y = ops.conv_dropout_bn(x, w, b, gamma, beta, mm, mv, True, 0.1, seed=4242, relu=True, stride=stride)
        else:
            u, _ = ops.conv2d(x, w, b, stride)
            u = ops.dropout(u, 0.1, True, seed=4242)
            y = ops.batch_norm(u, gamma, beta, mm, mv, True, relu=True)
        y.backward(gy)
        outs.append([y, x.grad, w.grad, b.grad, gamma.grad, beta.grad, mm, mv])
    for a, b in zip(*outs):
        assert rel(a, b) < 2e-3, rel(a, b)


def test_maxpool_dropout_bn_node(env, cuda):
    ops = env[0]
    N, H, W, C = 4, 16, 24, 64
    g = torch.Generator(device="cpu").manual_seed(7)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    gy = torch.randn((N, H // 2, W // 2, C), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(C, cuda, 8)
        if fused:
            y = ops.maxpool_dropout_bn(x, 2, 2, gamma, beta, mm, mv, True, 0.1, seed=55)
        else:
            u = ops.max_pool(x, 2, 2)
            u = ops.dropout(u, 0.1, True, seed=55)
            y = ops.batch_norm(u, gamma, beta, mm, mv, True, relu=True)
        y.backward(gy)
        outs.append([y, x.grad, gamma.grad, beta.grad, mm, mv])
    for a, b in zip(*outs):
        assert rel(a, b) < 2e-3, rel(a, b)


def test_residual_link(env, cuda):
    """BN(x) ... + x with a ResidualLink == plain autograd accumulation."""
    ops = env[0]
    N, H, W, C = 4, 8, 16, 64
    g = torch.Generator(device="cpu").manual_seed(9)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((C, 3, 3, C), generator=g) * 0.05).to(cuda)
    gz = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for linked in (False, True):
        x = x0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(C, cuda, 10)
        link = ops.ResidualLink() if linked else None
        y = ops.batch_norm(x, gamma, beta, mm, mv, True, relu=True, link=link)
        y, _ = ops.conv2d(y, w0, None)
        z, st = ops.add(y, x, relu=True, want_stats=True, link=link)
        z.backward(gz)
        outs.append([z, x.grad, gamma.grad, beta.grad, st.sum(0)])
    # x.grad: the linked path rounds (bn_dx + residual) once to bf16, autograd
    # rounds bn_dx first and the sum again -> one-ulp flips on many elements
    for i, (a, b) in enumerate(zip(*outs)):
        assert rel(a, b) < (5e-3 if i == 1 else 2e-3), (i, rel(a, b))


@pytest.mark.parametrize("C", [16, 64, 128])
def test_fused_channel_sums(env, cuda, C):
    """acfe_bn_bwd_apply_ex / acfe_relu_bwd_sum: the stored dx is bit-identical
    to the plain kernels and the fused per-channel sums equal channel_sum(dx)."""
    ops, call, lib, ptr, stream = env
    rows = 4000
    g = torch.Generator(device="cpu").manual_seed(11)
    dy = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    x = torch.randn((rows, C), generator=g).to(torch.bfloat16).to(cuda)
    scale, shift, coef = (torch.randn((n,), generator=g).to(cuda) for n in (C, C, 3 * C))
    nb = lib.acfe_reduce_blocks(rows)
    for rate in (0.0, 0.1):
        d0, d1 = torch.empty_like(x), torch.empty_like(x)
        call("acfe_bn_bwd_apply_dropout", ptr(dy), 1, ptr(x), 1, rows, C, ptr(scale), ptr(shift), 1, ptr(coef),
             rate, 5, ptr(d0), 1, stream())
        part = torch.empty((nb, 2, C), dtype=torch.float64, device=cuda)
        call("acfe_bn_bwd_apply_ex", ptr(dy), 1, ptr(x), 1, rows, C, ptr(scale), ptr(shift), 1, ptr(coef), None,
             rate, 5, ptr(d1), 1, ptr(part), stream())
        assert torch.equal(d0, d1)
        assert not part[:, 1].any()  # the sum-of-squares row is not formed (acfe.h)
        s = torch.empty((C,), device=cuda)
        call("acfe_channel_sum_finalize", ptr(part), nb, C, 0.0, ptr(s), stream())
        torch.testing.assert_close(s, ops.channel_sum(d0, C), rtol=1e-5, atol=1e-4)
    d0, d1 = torch.empty_like(x), torch.empty_like(x)
    call("acfe_relu_bwd", ptr(dy), ptr(x), dy.numel(), ptr(d0), 1, stream())
    part = torch.empty((nb, 2, C), dtype=torch.float64, device=cuda)
    call("acfe_relu_bwd_sum", ptr(dy), ptr(x), rows, C, ptr(d1), 1, ptr(part), stream())
    assert torch.equal(d0, d1)
    s = torch.empty((C,), device=cuda)
    call("acfe_channel_sum_finalize", ptr(part), nb, C, 0.0, ptr(s), stream())
    torch.testing.assert_close(s, ops.channel_sum(d0, C), rtol=1e-5, atol=1e-4)


def _c1bn_reference(x0, w0, b0, gamma, beta, mm, mv, gy, training, eps=1e-3, momentum=0.99):
    """float64 torch-CPU restatement of Conv2D(1x1) -> BatchNormalization (Keras:
    biased batch variance, moving averages with momentum) -> ReLU, on the
    bf16-rounded weights the kernels multiply with."""
    x = x0.double().cpu().requires_grad_(True)
    w = w0.to(torch.bfloat16).double().cpu().reshape(w0.shape[0], -1).requires_grad_(True)
    b = b0.double().cpu().requires_grad_(True)
    g = gamma.detach().double().cpu().requires_grad_(True)
    be = beta.detach().double().cpu().requires_grad_(True)
    a = x @ w.T + b
    if training:
        mean, var = a.mean((0, 1, 2)), a.var((0, 1, 2), unbiased=False)
    else:
        mean, var = mm.double().cpu(), mv.double().cpu()
    y = torch.relu(g * (a - mean) / torch.sqrt(var + eps) + be)
    y.backward(gy.double().cpu())
    mm1, mv1 = mm.double().cpu(), mv.double().cpu()
    if training:
        mm1 = mm1 * momentum + mean.detach() * (1 - momentum)
        mv1 = mv1 * momentum + var.detach() * (1 - momentum)
    return [y, x.grad, w.grad.reshape(w0.shape), g.grad, be.grad, mm1, mv1, b.grad]


@pytest.mark.parametrize("shape", [(3, 10, 37), (5, 128, 469)], ids=["ragged", "multi-pass"])
@pytest.mark.parametrize("K", [128, 64])
@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
def test_conv1x1_bn_node(env, cuda, shape, K, training):
    """The 1x1-conv + BN node (csrc/c1bn.hip: conv output never stored, its
    statistics from the Gram matrix of x, the backward sums from g^T x) and the
    unfused conv2d -> batch_norm chain, both against a float64 restatement: the
    fused node must be as accurate as the unfused chain (rel-L2 error at most
    1.25x the unfused error + 1e-3 on y, every gradient and the moving
    statistics).  In training mode the conv-bias gradient is zero in exact
    arithmetic: bounded absolutely.  'ragged': 1110 pixels (a partial last
    32-pixel chunk); 'multi-pass': 300160 pixels, several grid-stride passes
    per wave in every kernel."""
    ops = env[0]
    N, H, W = shape
    C = 16
    g = torch.Generator(device="cpu").manual_seed(12)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 1, 1, C), generator=g) * 0.2).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gy = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    gamma, beta, mm, mv = _bn_params(K, cuda, 13)
    ref = _c1bn_reference(x0, w0, b0, gamma, beta, mm, mv, gy, training)
    outs = []
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(K, cuda, 13)
        if fused:
            assert ops._c1bn_ok(x, w, 1)
            y = ops.conv_bn(x, w, b, gamma, beta, mm, mv, training, relu=True)
        else:
            u, st = ops.conv2d(x, w, b, 1, want_stats=training)
            y = ops.batch_norm(u, gamma, beta, mm, mv, training, relu=True, stats=st if training else None)
        y.backward(gy)
        outs.append([y, x.grad, w.grad, gamma.grad, beta.grad, mm, mv, b.grad])
    names = ["y", "dx", "dw", "dgamma", "dbeta", "moving_mean", "moving_var", "db"]
    for i in range(7):
        ef, eu = rel(outs[1][i], ref[i]), rel(outs[0][i], ref[i])
        assert ef <= 1.25 * eu + 1e-3, (names[i], ef, eu)
    if training:
        assert (outs[1][-1].double().cpu() - ref[-1]).norm().item() < 1e-3 * ref[2].norm().item()
    else:
        assert rel(outs[1][-1], ref[-1]) <= 1.25 * rel(outs[0][-1], ref[-1]) + 1e-3


@pytest.mark.parametrize("K,C", [(128, 128), (64, 64), (64, 128)])
def test_conv_pool_kernels(env, cuda, K, C):
    """Pooled-epilogue conv and its unpooling backward against the separate
    kernels, bit-exact: acfe_conv2d_fwd_pool == acfe_conv2d_fwd ->
    acfe_maxpool2d_fused (values, argmax bytes; statistics to 1e-6),
    acfe_conv2d_{dgrad,wgrad}_unpool == acfe_maxpool2d_bwd_argmax ->
    acfe_conv2d_{dgrad,wgrad}.  H = 14: the last 6-row tile is partly outside."""
    ops, call, lib, ptr, stream = env
    N, H, W = 2, 14, 128
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(21)
    x = torch.randn((N, H, W, C), generator=g).to(bf).to(cuda)
    w = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    b = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    assert lib.acfe_conv2d_pool_supported(N, H, W, C, K, 3, 3, 1) and lib.acfe_conv2d_pool_supported(N, H, W, K, C, 3,
                                                                                                        3, 1)
    wp = ops.pack_weights(w, bf, False)
    y0 = torch.empty((N, H, W, K), dtype=bf, device=cuda)
    call("acfe_conv2d_fwd", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y0), 1, None, stream())
    P, Q = H // 2, W // 2
    yp0 = torch.empty((N, P, Q, K), dtype=bf, device=cuda)
    am0 = torch.empty((N, P, Q, K), dtype=torch.uint8, device=cuda)
    st0 = torch.empty((lib.acfe_reduce_blocks(N * P * Q), 2, K), dtype=torch.float64, device=cuda)
    call("acfe_maxpool2d_fused", ptr(y0), N, H, W, K, 2, 2, ptr(yp0), ptr(am0), 0.1, 77, ptr(st0), 1, stream())
    yp1, am1 = torch.empty_like(yp0), torch.empty_like(am0)
    st1 = torch.empty((lib.acfe_conv2d_stats_rows(N * H * W, K), 2, wp.shape[0]), dtype=torch.float64, device=cuda)
    call("acfe_conv2d_fwd_pool", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(yp1), ptr(am1), 0.1, 77, ptr(st1),
         1, stream())
    assert torch.equal(yp1, yp0)
    assert torch.equal(am1, am0)
    torch.testing.assert_close(st1.sum(0)[:, :K], st0.sum(0), rtol=1e-6, atol=1e-4)
    # backward from a pooled gradient
    gp = torch.randn((N, P, Q, K), generator=g).to(bf).to(cuda)
    dfull = torch.empty((N, H, W, K), dtype=bf, device=cuda)
    call("acfe_maxpool2d_bwd_argmax", ptr(am0), ptr(gp), N, H, W, K, 2, 2, 0.0, 0, ptr(dfull), 1, stream())
    wf = ops.pack_weights(w, bf, True)
    dx0, dx1 = (torch.empty((N, H, W, C), dtype=bf, device=cuda) for _ in range(2))
    call("acfe_conv2d_dgrad", ptr(dfull), N, H, W, K, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx0), 1, None, stream())
    call("acfe_conv2d_dgrad_unpool", ptr(gp), ptr(am0), N, H, W, K, ptr(wf), C, 1, 1, ptr(dx1), 1, stream())
    assert torch.equal(dx1, dx0)
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)
    dw0, dw1 = (torch.empty((K, 3, 3, C), device=cuda) for _ in range(2))
    call("acfe_conv2d_wgrad", ptr(x), N, H, W, C, ptr(dfull), K, 3, 3, 1, 1, 1, H, W, ptr(dw0), 0.0, 1, ptr(ws),
         stream())
    call("acfe_conv2d_wgrad_unpool", ptr(x), N, H, W, C, ptr(gp), ptr(am0), K, 1, 1, ptr(dw1), 0.0, 1, ptr(ws),
         stream())
    assert torch.equal(dw1, dw0)


def test_conv_maxpool_dropout_bn_node(env, cuda):
    """The pooled-epilogue node against conv2d -> maxpool_dropout_bn (same
    dropout seed): outputs and every gradient within rel-L2 2e-3."""
    ops = env[0]
    N, H, W, C, K = 3, 16, 64, 64, 64
    g = torch.Generator(device="cpu").manual_seed(22)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gy = torch.randn((N, H // 2, W // 2, K), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(K, cuda, 23)
        if fused:
            assert ops._conv_pool_ok(x, w, 1, "same", 2, 2)
            y = ops.conv_maxpool_dropout_bn(x, w, b, 1, "same", 2, 2, gamma, beta, mm, mv, True, 0.1, seed=99)
        else:
            u, _ = ops.conv2d(x, w, b, 1)
            y = ops.maxpool_dropout_bn(u, 2, 2, gamma, beta, mm, mv, True, 0.1, seed=99)
        y.backward(gy)
        outs.append([y, x.grad, w.grad, b.grad, gamma.grad, beta.grad, mm, mv])
    for i, (a, r) in enumerate(zip(outs[1], outs[0])):
        assert rel(a, r) < 2e-3, (i, rel(a, r))


def test_pool_link(env, cuda):
    """BN(x) ... + Conv(AvgPool(x)) with the pooled shortcut gradient folded into
    the BN backward (acfe_bn_bwd_apply_pool via ResidualLink) == plain autograd
    accumulation of the AveragePooling2D backward; the input being a ReLU output
    also folds that ReLU's backward in (relu flag bit 1)."""
    ops = env[0]
    N, H, W, C = 4, 10, 18, 16  # odd pooled extents are not needed: H, W even as in the model
    g = torch.Generator(device="cpu").manual_seed(31)
    a0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    b0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((32, 1, 1, C), generator=g) * 0.2).to(cuda)
    gz = torch.randn((N, H // 2, W // 2, 32), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for linked in (False, True):
        a, b = a0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        gamma, beta, mm, mv = _bn_params(C, cuda, 32)
        x = ops.add(a, b, relu=True)  # ReLU output: its backward folds into the BN
        link = ops.ResidualLink() if linked else None
        u = ops.batch_norm(x, gamma, beta, mm, mv, True, relu=True, link=link)
        u, _ = ops.conv2d(ops.avg_pool_same(u, 2), w0, None)
        s, _ = ops.conv2d(ops.avg_pool_same(x, 2, link=link), w0, None)
        z = ops.add(u, s)
        z.backward(gz)
        outs.append([z, a.grad, b.grad, gamma.grad, beta.grad])
    for i, (p, r) in enumerate(zip(outs[1], outs[0])):
        assert rel(p, r) < (5e-3 if i in (1, 2) else 2e-3), (i, rel(p, r))


@pytest.mark.parametrize("k,H,W", [(2, 16, 33), (3, 22, 31), (2, 12, 20)])
@pytest.mark.parametrize("relu", [1, 3])
def test_bn_bwd_apply_sub_bitexact(env, cuda, k, H, W, relu):
    """acfe_bn_bwd_apply_sub (the 1x1 stride-k shortcut's dX at the pixels
    (k p, k q) only) == acfe_bn_bwd_apply_ex with that gradient scattered into
    a zero tensor as `add`: dx bit-identical, channel sums equal."""
    ops, call, lib, ptr, stream = env
    N, C = 2, 64
    P, Q = (H - 1) // k + 1, (W - 1) // k + 1
    g = torch.Generator(device="cpu").manual_seed(17 + k)
    BF = torch.bfloat16
    dy = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    gs = torch.randn((N, P, Q, C), generator=g).to(BF).to(cuda)
    sc = (torch.rand((C,), generator=g) + 0.5).to(cuda)
    sh = (torch.randn((C,), generator=g) * 0.2).to(cuda)
    coef = (torch.randn((3 * C,), generator=g) * 0.5).to(cuda)
    full = torch.zeros((N, H, W, C), dtype=BF, device=cuda)
    full[:, ::k, ::k, :] = gs
    rows = N * H * W
    nb = lib.acfe_reduce_blocks(rows)
    outs = []
    for mode in ("ex", "sub"):
        dx = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
        sums = torch.empty((nb, 2, C), dtype=torch.float64, device=cuda)
        if mode == "ex":
            call("acfe_bn_bwd_apply_ex", ptr(dy), 1, ptr(x), 1, rows, C, ptr(sc), ptr(sh), relu, ptr(coef), ptr(full),
                 0.0, 0, ptr(dx), 1, ptr(sums), stream())
        else:
            call("acfe_bn_bwd_apply_sub", ptr(dy), 1, ptr(x), 1, N, H, W, C, ptr(sc), ptr(sh), relu, ptr(coef),
                 ptr(gs), k, ptr(dx), 1, ptr(sums), stream())
        torch.cuda.synchronize()
        outs.append((dx, sums[:, 0].sum(0)))
    assert torch.equal(outs[1][0].view(torch.int16), outs[0][0].view(torch.int16))
    assert torch.equal(outs[1][1], outs[0][1])


@pytest.mark.parametrize("k", [2, 3])
def test_sub_link_node(env, cuda, k):
    """wr_resnet's transition block shape (resnet/wr_resnet.py:46-90):
    BN(x) -> 3x3 conv stride k, plus a 1x1 "valid" stride-k conv shortcut of x
    whose dX reaches bn(x)'s backward through the ResidualLink at P x Q
    (acfe_bn_bwd_apply_sub) == the shortcut's full-resolution dX handed over
    (ACFE_SUB_FUSE=0 path) and == plain autograd accumulation."""
    ops = env[0]
    N, H, W, C, K = 2, 12 * k, 10 * k + 1, 64, 128
    g = torch.Generator(device="cpu").manual_seed(23 + k)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    ws0 = (torch.randn((K, 1, 1, C), generator=g) * 0.1).to(cuda)
    P = -(-H // k)
    Q = -(-W // k)
    gz = torch.randn((N, P, Q, K), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    old = ops.FUSE_SUB
    try:
        for mode in ("autograd", "full", "sub"):
            ops.FUSE_SUB = mode == "sub"
            x = x0.clone().requires_grad_(True)
            w, ws = w0.clone().requires_grad_(True), ws0.clone().requires_grad_(True)
            gamma, beta, mm, mv = _bn_params(C, cuda, 29)
            link = None if mode == "autograd" else ops.ResidualLink()
            u = ops.batch_norm(x, gamma, beta, mm, mv, True, relu=True, link=link)
            y, _ = ops.conv2d(u, w, None, k, "same")
            s, _ = ops.conv2d(x, ws, None, k, "valid", link=link)
            z = ops.add(y, s)
            z.backward(gz)
            outs.append([z, x.grad, w.grad, ws.grad, gamma.grad, beta.grad])
    finally:
        ops.FUSE_SUB = old
    for i, (a, b) in enumerate(zip(outs[2], outs[1])):  # sub vs full hand-over: same arithmetic
        assert rel(a, b) < 1e-6, ("full", i, rel(a, b))
    for i, (a, b) in enumerate(zip(outs[2], outs[0])):
        assert rel(a, b) < 2e-3, ("autograd", i, rel(a, b))


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("C,K", [(64, 64), (128, 64), (64, 128), (32, 128), (16, 256), (32, 256), (128, 128),
                                 (256, 256), (128, 256)])
def test_conv_add_node(env, cuda, relu, C, K):
    """(ReLU)(conv 3x3 + shortcut) with the Add in the conv epilogue
    (acfe_conv2d_fwd_add: the rows kernel -- K = C = 128: the one-wave
    k_conv3x3_1w<3> --, for the stage-2/3 conv2b shapes C = 16 / 32,
    K = 128 / 256 the generic kernel with the Add in its row stores, for
    wr_resnet's 256-channel stage 3 the persistent GEMM k_conv_fwd_p<RES>) ==
    conv2d -> add: z bit-exact, statistics to 1e-6, gradients of x,
    w, b and the shortcut identical up to summation order."""
    ops = env[0]
    N, H, W = 2, 14, 128
    g = torch.Generator(device="cpu").manual_seed(41)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    s0 = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gz = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    for fused in (False, True):
        x, s = x0.clone().requires_grad_(True), s0.clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        if fused:
            assert ops._conv_add_ok(x, w, s, 1, "same")
            z, st = ops.conv_add(x, w, b, s, relu=relu, want_stats=True)
        else:
            y, _ = ops.conv2d(x, w, b)
            z, st = ops.add(y, s, relu=relu, want_stats=True)
        z.backward(gz)
        outs.append([z, st.sum(0)[:, :K], x.grad, w.grad, b.grad, s.grad])
    assert torch.equal(outs[1][0], outs[0][0])
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=1e-6, atol=1e-4)
    for i in range(2, 6):
        assert rel(outs[1][i], outs[0][i]) < 1e-3, (i, rel(outs[1][i], outs[0][i]))


@pytest.mark.parametrize("mode", ["single", "opt_out", "second_consumer"])
def test_conv_add_bn_fold_consumers(env, cuda, mode):
    """The BN-backward fold into conv_add's weight gradient is opt-in
    (single_consumer=True): with one BN consumer the folded
    gradients equal the unfused chain; without the opt-in a second consumer of
    z (a BN and another op) gets correct gradients; opted in while z has a
    second consumer, the backward raises instead of reading unwritten memory."""
    ops = env[0]
    N, H, W, C, K = 2, 14, 128, 64, 64
    g = torch.Generator(device="cpu").manual_seed(43)
    x0 = torch.randn((N, H, W, C), generator=g).to(torch.bfloat16).to(cuda)
    s0 = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 3, 3, C), generator=g) * 0.05).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gy = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    gamma0 = (1 + 0.2 * torch.randn(K, generator=g)).to(cuda)
    beta0 = (0.1 * torch.randn(K, generator=g)).to(cuda)

    def run(fused, single, second):
        x = x0.clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        gamma, beta = gamma0.clone().requires_grad_(True), beta0.clone().requires_grad_(True)
        mm, mv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
        if fused:
            z, st = ops.conv_add(x, w, b, s0, relu=True, want_stats=True, single_consumer=single)
        else:
            y, _ = ops.conv2d(x, w, b)
            z, st = ops.add(y, s0, relu=True, want_stats=True)
        out = ops.batch_norm(z, gamma, beta, mm, mv, True, relu=True, stats=st)
        loss = (out.float() * gy.float()).sum()
        if second:
            loss = loss + (z.float() * 0.5).sum()
        loss.backward()
        return [x.grad, w.grad, b.grad, gamma.grad, beta.grad]

    if mode == "second_consumer":
        with pytest.raises(RuntimeError, match="pending"):
            run(True, True, True)
        return
    second = mode == "opt_out"
    ref = run(False, False, second)
    got = run(True, mode == "single", second)
    for i, (a, r) in enumerate(zip(got, ref)):
        assert torch.isfinite(a).all()
        assert rel(a, r) < 2e-3, (i, rel(a, r))


@pytest.mark.parametrize("W", [66, 67])
@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
def test_bn_maxpool_node(env, cuda, training, dtype, W, monkeypatch):
    """MaxPool2D((1, 2))(BatchNormalization(x)) with the BN formed at load time
    inside the pooling kernel (acfe_bn_maxpool2d_fused) == batch_norm -> max_pool:
    pooled output bit-exact, statistics of it to 1e-6, gradients of x, gamma
    and beta identical up to summation order."""
    ops = env[0]
    N, H, C = 2, 16, 16  # odd W: the last column is dropped by the pooling
    g = torch.Generator(device="cpu").manual_seed(7)
    x0 = (torch.randn((N, H, W, C), generator=g) * 2 + 0.3).to(dtype).to(cuda)
    gamma0 = (1 + 0.2 * torch.randn(C, generator=g)).to(cuda)
    beta0 = (0.1 * torch.randn(C, generator=g)).to(cuda)
    mm0 = (0.1 * torch.randn(C, generator=g)).to(cuda)
    mv0 = (1 + torch.rand(C, generator=g)).to(cuda)
    gy = torch.randn((N, H, W // 2, C), generator=g).to(dtype).to(cuda)
    outs = []
    for fuse in (False, True):
        monkeypatch.setattr(ops, "FUSE", fuse)
        x = x0.clone().requires_grad_(True)
        gamma, beta = gamma0.clone().requires_grad_(True), beta0.clone().requires_grad_(True)
        mm, mv = mm0.clone(), mv0.clone()
        y, st = ops.bn_max_pool(x, gamma, beta, mm, mv, training, 1, 2, want_stats=training)
        y.backward(gy)
        outs.append([y, st, x.grad, gamma.grad, beta.grad, mm, mv])
    assert torch.equal(outs[1][0], outs[0][0])
    if training:
        torch.testing.assert_close(outs[1][1].sum(0), outs[0][1].sum(0), rtol=1e-6, atol=1e-4)
        assert torch.equal(outs[1][5], outs[0][5]) and torch.equal(outs[1][6], outs[0][6])
    for i in (2, 3, 4):
        assert rel(outs[1][i], outs[0][i]) < 1e-5, (i, rel(outs[1][i], outs[0][i]))


@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("shape", [(3, 10, 37), (4, 64, 128)], ids=["ragged", "stage1"])
def test_bn_prologue_conv1x1_bn_node(env, cuda, shape, training):
    """bn2a0 -> ReLU -> (1x1 conv + BN node) with the first BN handed to the node
    as a prologue (its output pending, never written: acfe_c1bn_*_bn) against
    the same chain with the BN output written by acfe_bn_apply: bit-identical
    output, input gradient, weight / bias / BN-parameter gradients and moving
    statistics (resnet/wr_resnet_bird.py:121-131)."""
    ops = env[0]
    N, H, W = shape
    C, K = 16, 128
    g = torch.Generator(device="cpu").manual_seed(21)
    x0 = (torch.randn((N, H, W, C), generator=g) * 2 + 0.3).to(torch.bfloat16).to(cuda)
    w0 = (torch.randn((K, 1, 1, C), generator=g) * 0.2).to(cuda)
    b0 = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    gy = torch.randn((N, H, W, K), generator=g).to(torch.bfloat16).to(cuda)
    outs = []
    saved = ops.PRO_C1
    ops.PRO_C1 = True  # (off by default in the model: measured slower)
    try:
        for defer in (False, True):
            x = x0.clone().requires_grad_(True)
            w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
            ga, ba, ma, va = _bn_params(C, cuda, 31)
            gb, bb, mb, vb = _bn_params(K, cuda, 32)
            xb = ops.batch_norm(x, ga, ba, ma, va, training, relu=True, defer=defer)
            assert (ops._pending(xb) is not None) == defer
            y = ops.conv_bn(xb, w, b, gb, bb, mb, vb, training, relu=True)
            assert (ops._pending(xb) is not None) == defer  # the node never writes it
            y.backward(gy)
            outs.append([y, x.grad, w.grad, b.grad, ga.grad, ba.grad, gb.grad, bb.grad, ma, va, mb, vb])
    finally:
        ops.PRO_C1 = saved
    names = ["y", "dx", "dw", "db", "dgamma_a", "dbeta_a", "dgamma_b", "dbeta_b", "mm_a", "mv_a", "mm_b", "mv_b"]
    for n, a, b in zip(names, outs[0], outs[1]):
        assert torch.equal(a, b), n
