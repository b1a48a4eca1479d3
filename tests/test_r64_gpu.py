"""Parity of the K = 64 row-halo convolutions with the interleaved epilogue
(k_conv3x3_r64, csrc/rows64.hip) against the kernel it
replaces (k_conv3x3_rows<64, 8, PM, true>) AND against float64.

The new kernel computes every accumulator with the same MFMA sequence and the
same epilogue arithmetic (bias, bf16 rounding, the pair-hash dropout, the
residual Add + ReLU, the BN sums in the same per-lane order over the same
persistent tile walk), so every output -- y, the BN statistics slab, the
prologue's x', the dgrad's dX and its BN-backward-reduce slab -- must be BIT
IDENTICAL to the previous kernel (acfe_conv_r64_enable(0)).  The float64
check guards against a defect shared by both: y within one bf16 ulp of the
exact conv of the same bf16 operands.  Shapes: full 8 x 64 tiles, ragged
images (a partial last row tile and 64-column tile), C = 64 / 128 / 256
input channels (1 / 2 / 4 chunks per tile), at tile counts where every
workgroup walks several tiles (the inter-tile epilogue runs), and one
workgroup with a single tile.

Images whose width is not a multiple of 64 (wr_resnet's 513-wide stage 1) run
their Q % 64 last pixels of each row as a second launch of 32 x 16 tiles
(r06): y, x' and dX stay bit-identical, while the statistics slabs then hold
other per-workgroup partial sums -- their column sums are compared to 1e-6
relative (each tile's values are summed in f32 before the f64 slab, so other
tiles give other f32 roundings; + 1e-3 for the cancelling dgrad reduce sums)."""
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
    e = torch.floor(torch.log2(t.abs().clamp_min(2.0 ** -120)))
    return torch.pow(2.0, e - 7)


def _within_ulp(gpu, exact, atol=1e-4, what=""):
    g = gpu.detach().to(F64).cpu()
    err = (g - exact).abs()
    nbad = int((err > _ulp(exact) + atol).sum())
    assert nbad == 0, (what, nbad, float(err.max()))


def _both(lib, fn):
    """fn() under the previous kernel and under k_conv3x3_r64."""
    prev = lib.acfe_conv_r64_enable(0)
    try:
        a = fn()
        lib.acfe_conv_r64_enable(1)
        b = fn()
    finally:
        lib.acfe_conv_r64_enable(prev)
    torch.cuda.synchronize()
    return a, b


def _same(a, b, what):
    for i, (x, y) in enumerate(zip(a, b)):
        if x is None:
            continue
        if x.dtype == F64:  # a statistics slab: per-channel totals over its rows
            sx, sy = x.sum(0), y.sum(0)
            assert ((sx - sy).abs() <= 1e-6 * sx.abs() + 1e-3).all(), (what, i)
            continue
        if x.dtype == BF:
            x, y = x.view(torch.int16), y.view(torch.int16)
        assert torch.equal(x, y), (what, i, (x.float() - y.float()).abs().max().item())


SHAPES = [(16, 16, 128, 64), (3, 13, 100, 64), (2, 9, 70, 128), (12, 16, 128, 128), (4, 16, 64, 256),
          (1, 8, 64, 64), (3, 40, 129, 64)]


@pytest.mark.parametrize("N,H,W,C", SHAPES, ids=[f"{n}x{h}x{w}c{c}" for n, h, w, c in SHAPES])
@pytest.mark.parametrize("mode", ["plain", "plain_stats", "drop", "bn_drop", "bn_plain", "add", "add_norelu",
                                  "add_bn", "add_nostats"])
def test_r64_forward(env, cuda, N, H, W, C, mode):
    ops, call, lib, ptr, stream = env
    K = 64
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + H * 10 + C)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    w = (torch.randn((K, 3, 3, C), generator=g) * (1.0 / (3 * C ** 0.5))).to(cuda)
    b = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    res = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    sc = ((torch.rand(C, generator=g) * 1.5 + 0.25) * torch.where(torch.rand(C, generator=g) < 0.1, -1.0, 1.0)).to(cuda)
    sh = (torch.randn(C, generator=g) * 0.5).to(cuda)
    wp = ops.pack_weights(w, BF, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    pro = mode.startswith("bn") or mode == "add_bn"

    def run():
        y = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
        st = torch.full((rows, 2, wp.shape[0]), float("nan"), dtype=F64, device=cuda)
        xb = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda) if pro else None
        if mode in ("plain", "plain_stats", "drop"):
            rate = 0.1 if mode == "drop" else 0.0
            stp = None if mode == "plain" else ptr(st)
            call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y), 1,
                 stp, rate, 77, stream())
        elif mode in ("bn_drop", "bn_plain"):
            rate = 0.1 if mode == "bn_drop" else 0.0
            call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), rate, 78,
                 ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
        elif mode == "add_bn":
            call("acfe_conv2d_fwd_add_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(res), 1, ptr(y),
                 ptr(st), ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
        else:
            relu = 0 if mode == "add_norelu" else 1
            stp = None if mode == "add_nostats" else ptr(st)
            call("acfe_conv2d_fwd_add", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(res), relu, ptr(y), stp, 1,
                 stream())
        has_st = mode not in ("plain", "add_nostats")
        return [y, st[:, :, :K] if has_st else None, xb]

    a, bb = _both(lib, run)
    _same(a, bb, mode)
    y = bb[0]
    assert not torch.isnan(y.float()).any()
    # float64 check of the conv part (before dropout / residual): the plain modes
    if mode in ("plain", "plain_stats", "bn_plain"):
        xin = bb[2] if pro else x
        xe = xin.detach().cpu().to(F64).permute(0, 3, 1, 2)
        we = w.detach().cpu().to(BF).to(F64).permute(0, 3, 1, 2)
        exact = F.conv2d(xe, we, b.detach().cpu().to(F64), padding=1).permute(0, 2, 3, 1)
        _within_ulp(y, exact, what=mode)
    if bb[1] is not None:
        s = bb[1].sum(0).cpu()
        t = y.detach().to(F64).cpu().reshape(-1, K)
        ref = torch.stack([t.sum(0), (t * t).sum(0)])
        assert ((s - ref).abs() <= 1e-6 * ref.abs().clamp_min(1.0) + 1e-3).all(), mode


@pytest.mark.parametrize("N,H,W,Kd", [(16, 16, 128, 64), (3, 13, 100, 64), (2, 9, 70, 128), (4, 16, 64, 256),
                                     (3, 40, 129, 64)],
                         ids=["full", "ragged", "k128", "k256", "w129"])
@pytest.mark.parametrize("relu", [1, 0])
def test_r64_dgrad(env, cuda, N, H, W, Kd, relu):
    """acfe_conv2d_dgrad (stride 1, 64 dX channels) and acfe_conv2d_dgrad_bn
    (the BN backward reduce slab in the epilogue) from Kd dY channels."""
    ops, call, lib, ptr, stream = env
    C = 64
    g = torch.Generator(device="cpu").manual_seed(N * 77 + Kd + relu)
    dy = torch.randn((N, H, W, Kd), generator=g).to(BF).to(cuda)
    w = (torch.randn((Kd, 3, 3, C), generator=g) * (1.0 / (3 * C ** 0.5))).to(cuda)
    xb = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    sc = (torch.rand(C, generator=g) + 0.5).to(cuda)
    sh = (torch.randn(C, generator=g) * 0.3).to(cuda)
    mu = (torch.randn(C, generator=g) * 0.1).to(cuda)
    inv = (torch.rand(C, generator=g) + 0.5).to(cuda)
    wf = ops.pack_weights(w, BF, True)
    brows = lib.acfe_conv2d_dgrad_bn_rows(N, H, W, C, Kd, 3, 3, 1, 1)
    assert brows > 0

    def run():
        dx0 = torch.full((N, H, W, C), float("nan"), dtype=BF, device=cuda)
        dx1 = torch.full_like(dx0, float("nan"))
        part = torch.full((brows, 2, C), float("nan"), dtype=F64, device=cuda)
        call("acfe_conv2d_dgrad", ptr(dy), N, H, W, Kd, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx0), 1, None,
             stream())
        call("acfe_conv2d_dgrad_bn", ptr(dy), N, H, W, Kd, ptr(wf), C, 3, 3, 1, 1, 1, H, W, ptr(dx1), 1, ptr(xb),
             ptr(sc), ptr(sh), ptr(mu), ptr(inv), relu, ptr(part), brows, stream())
        return [dx0, dx1, part]

    a, b = _both(lib, run)
    _same(a, b, "dgrad")
    assert torch.equal(b[0].view(torch.int16), b[1].view(torch.int16))
    gd = dy.detach().cpu().to(F64).permute(0, 3, 1, 2)
    wd = w.detach().cpu().to(BF).to(F64).permute(0, 3, 1, 2)
    _within_ulp(b[0], F.conv_transpose2d(gd, wd, padding=1).permute(0, 2, 3, 1), what="dX")
    # the slab: acfe_bn_bwd_reduce's sums of the stored dX
    d = b[1].detach().cpu().to(F64).reshape(-1, C)
    xv = xb.detach().cpu().to(F64).reshape(-1, C)
    m = torch.ones_like(d) if not relu else ((xv * sc.cpu().to(F64) + sh.cpu().to(F64)) > 0).to(F64)
    gm = d * m
    ref = torch.stack([gm.sum(0), (gm * (xv - mu.cpu().to(F64)) * inv.cpu().to(F64)).sum(0)])
    s = b[2].sum(0).cpu()
    assert ((s - ref).abs() <= 1e-5 * ref.abs().clamp_min(1.0) + 1e-2).all()


@pytest.mark.parametrize("C,pro", [(64, False), (64, True), (128, True)], ids=["c64", "c64-bn", "c128-bn"])
def test_keep_bits(env, cuda, C, pro):
    """The dropout keep bits (acfe_conv2d_fwd_dropout_keep / _bn_keep): the
    forward's outputs are bit-identical to the forward without them, the bits
    are acfe_dropout's mask of the same (rate, seed, element index), and the
    BN-fold weight gradient reading them (acfe_conv2d_wgrad_bnbwd_keep) is
    bit-identical to the one regenerating the mask -- dY, dW and the slab."""
    ops, call, lib, ptr, stream = env
    N, H, W, K = 6, 14, 100, 64  # (the fold wgrad takes row pairs: even H; a partial 64-column tile)
    assert lib.acfe_conv2d_dropout_keep_supported(N, H, W, C, K, 1)
    g = torch.Generator(device="cpu").manual_seed(C + pro)
    x = torch.randn((N, H, W, C), generator=g).to(BF).to(cuda)
    w = (torch.randn((K, 3, 3, C), generator=g) * (1.0 / (3 * C ** 0.5))).to(cuda)
    b = (torch.randn((K,), generator=g) * 0.1).to(cuda)
    sc, sh = (torch.rand(C, generator=g) + 0.5).to(cuda), (torch.randn(C, generator=g) * 0.3).to(cuda)
    wp = ops.pack_weights(w, BF, False)
    rows = lib.acfe_conv2d_stats_rows(N * H * W, K)
    rate, seed = 0.1, 4242

    def fwd(keep):
        y = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
        st = torch.zeros((rows, 2, wp.shape[0]), dtype=F64, device=cuda)
        xb = torch.empty_like(x)
        if pro:
            if keep is None:
                call("acfe_conv2d_fwd_bn", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), rate, seed,
                     ptr(sc), ptr(sh), 1, ptr(xb), 1, stream())
            else:
                call("acfe_conv2d_fwd_bn_keep", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st), rate,
                     seed, ptr(sc), ptr(sh), 1, ptr(xb), ptr(keep), 1, stream())
        else:
            if keep is None:
                call("acfe_conv2d_fwd_dropout", ptr(x), N, H, W, C, ptr(wp), K, 3, 3, 1, 1, 1, H, W, ptr(b), ptr(y),
                     1, ptr(st), rate, seed, stream())
            else:
                call("acfe_conv2d_fwd_dropout_keep", ptr(x), N, H, W, C, ptr(wp), K, 1, 1, ptr(b), ptr(y), ptr(st),
                     rate, seed, ptr(keep), stream())
        torch.cuda.synchronize()
        return y, st
    keep = torch.full((N, H, W, K // 8), 0xAA, dtype=torch.uint8, device=cuda)
    y0, st0 = fwd(None)
    y1, st1 = fwd(keep)
    assert torch.equal(y1.view(torch.int16), y0.view(torch.int16)) and torch.equal(st1, st0)
    ones = torch.ones((N, H, W, K), dtype=BF, device=cuda)
    m = torch.empty_like(ones)
    call("acfe_dropout", ptr(ones), ones.numel(), rate, seed, ptr(m), 1, stream())
    torch.cuda.synchronize()
    mask = (m != 0).reshape(N, H, W, K // 8, 8).to(torch.int32)
    bits = sum(mask[..., j] << j for j in range(8)).to(torch.uint8)
    assert torch.equal(keep, bits)
    # the fold wgrad: BN backward apply (+ReLU mask) -> dropout backward inside the wgrad staging
    dy = torch.randn((N, H, W, K), generator=g).to(BF).to(cuda)
    u = y1
    bsc, bsh = (torch.rand(K, generator=g) + 0.5).to(cuda), (torch.randn(K, generator=g) * 0.2).to(cuda)
    coef = (torch.randn(3 * K, generator=g) * 0.3).to(cuda)
    brows = lib.acfe_conv2d_wgrad_bnbwd_rows(N, H, W, C, K)
    assert brows > 0
    ws = torch.empty((lib.acfe_conv2d_wgrad_workspace(N, H, W, C, K, 3, 3, H, W),), device=cuda)

    def fold(kp):
        gout = torch.full((N, H, W, K), float("nan"), dtype=BF, device=cuda)
        dw = torch.empty((K, 3, 3, C), device=cuda)
        sums = torch.empty((brows, 2, K), dtype=F64, device=cuda)
        if kp is None:
            call("acfe_conv2d_wgrad_bnbwd", ptr(x), N, H, W, C, ptr(dy), ptr(u), K, ptr(bsc), ptr(bsh), 1, ptr(coef),
                 None, rate, seed, ptr(gout), ptr(dw), 0.0, ptr(ws), ptr(sums), stream())
        else:
            call("acfe_conv2d_wgrad_bnbwd_keep", ptr(x), N, H, W, C, ptr(dy), ptr(u), K, ptr(bsc), ptr(bsh), 1,
                 ptr(coef), rate, seed, ptr(kp), ptr(gout), ptr(dw), 0.0, ptr(ws), ptr(sums), stream())
        torch.cuda.synchronize()
        return gout, dw, sums
    a, bb = fold(None), fold(keep)
    assert torch.equal(a[0].view(torch.int16), bb[0].view(torch.int16)), "dY"
    assert torch.equal(a[1], bb[1]) and torch.equal(a[2], bb[2])
