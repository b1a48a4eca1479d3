"""GPU parity of the fused front end (HIP, via the C ABI) against the CPU oracle.

Tolerances (fp32 kernels vs float64 oracle):
  mel:   |gpu - ref| <= 2e-5 * max(ref) per clip  (fp32 FFT, 11 passes)
  PCEN:  |gpu - ref| <= 5e-5 on the [-1, 1] output
  dPCEN: relative 2e-3 on parameter gradients (fp32 accumulation over B*M*T)
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, synth_clips
from oracle import frontend as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fe(cuda):
    from acfe import frontend

    return frontend


def _plan(fe, **kw):
    return fe.MelPlan(**kw)


def _rel_close(gpu, ref, tol):
    gpu = np.asarray(gpu, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).reshape(ref.shape[0], -1).max(1).reshape((-1,) + (1,) * (ref.ndim - 1))
    err = np.abs(gpu - ref) / scale
    assert err.max() <= tol, f"max rel err {err.max():.3e} > {tol}"
    return err.max()


def test_normalize_and_mixup(fe, cuda):
    x1 = torch.from_numpy(synth_clips(3, seed=11)).to(cuda)
    x2 = torch.from_numpy(synth_clips(3, seed=21)).to(cuda)
    y = fe.normalize(x1).cpu().numpy()
    np.testing.assert_allclose(y, of.normalize(x1.cpu().numpy()), atol=2e-6)
    lam = torch.tensor([0.0, 0.3, 0.9], device=cuda)
    st1, st2 = fe.normalize_stats(x1), fe.normalize_stats(x2)
    m = fe.mix_up(x1, x2, lam, st1, st2).cpu().numpy()
    ref, _ = of.mix_up(of.normalize(x1.cpu().numpy()), np.zeros((3, 2)), of.normalize(x2.cpu().numpy()),
                       np.zeros((3, 2)), lam.cpu().numpy())
    np.testing.assert_allclose(m, ref, atol=4e-6)


@pytest.mark.parametrize("n_mels,n_fft", [(128, 4096), (160, 4096), (96, 1024)])
def test_mel_pad_end(fe, cuda, n_mels, n_fft):
    raw = synth_clips(3, seed=5)
    plan = _plan(fe, n_mels=n_mels, n_fft=n_fft)
    x = torch.from_numpy(raw).to(cuda)
    st = fe.normalize_stats(x)
    out = plan.mel(x, st, pad_mode="end", layout="btm").cpu().numpy()
    ref = of.raw_to_mel(of.normalize(raw), plan.weights, n_fft, 281).transpose(0, 2, 1)
    assert out.shape == ref.shape == (3, 513, n_mels)
    _rel_close(out, ref, 2e-5)
    bmt = plan.mel(x, st, pad_mode="end", layout="bmt").cpu().numpy()
    np.testing.assert_array_equal(bmt, out.transpose(0, 2, 1))


@pytest.mark.parametrize("pad_mode", ["constant", "reflect"])
def test_mel_center_predict_path(fe, cuda, pad_mode):
    raw = synth_clips(2, seed=7)
    plan = _plan(fe, n_mels=160)
    x = torch.from_numpy(raw).to(cuda)
    out = plan.mel(x, fe.normalize_stats(x), pad_mode=pad_mode, layout="bmt").cpu().numpy()
    ref = of.get_spect(of.normalize(raw), plan.weights, 4096, 281, 2, pad_mode)
    _rel_close(out, ref, 2e-5)


def test_mel_power1_no_norm(fe, cuda):
    raw = synth_clips(2, seed=8) * 0.5
    plan = _plan(fe)
    out = plan.mel(torch.from_numpy(raw).to(cuda), None, power=1, layout="bmt").cpu().numpy()
    ref = of.raw_to_mel(raw, plan.weights, 4096, 281, power=1)
    _rel_close(out, ref, 2e-5)


def test_mel_streaming_windows(fe, cuda):
    """Overlapping 3 s windows at a 1.5 s hop of one recording (clip_stride < n)."""
    rec = synth_clips(1, n=48000 * 9, seed=9)[0]
    plan = _plan(fe)
    x = torch.from_numpy(rec).to(cuda)
    nwin = 1 + (len(rec) - 144000) // 72000
    st = fe.normalize_stats(x, n=144000, clip_stride=72000, batch=nwin)
    out = plan.mel(x, st, pad_mode="constant", layout="bmt", n=144000, clip_stride=72000, batch=nwin).cpu().numpy()
    wins = np.stack([rec[i * 72000: i * 72000 + 144000] for i in range(nwin)])
    ref = of.get_spect(of.normalize(wins), plan.weights, 4096, 281, 2, "constant")
    _rel_close(out, ref, 2e-5)


@pytest.mark.parametrize("n_mels,pad_mode,norm,power", [(128, "end", True, 2), (160, "constant", True, 2),
                                                        (128, "reflect", False, 1), (40, "end", True, 2)])
def test_mel_kernel_modes(fe, cuda, n_mels, pad_mode, norm, power):
    """k_mel_w4 across its modes against the float64 oracle: normalise-on-load
    (stats) or raw input, the three framings (padded boundary frames), power 1
    and 2, and a plan whose bins do not fill a thread round (40 mels up to
    1.5 kHz)."""
    raw = synth_clips(3, seed=17)
    fmax = 11000 if n_mels != 40 else 1500
    plan = _plan(fe, n_mels=n_mels, fmax=fmax)
    x = torch.from_numpy(raw).to(cuda)
    st = fe.normalize_stats(x) if norm else None
    out = plan.mel(x, st, pad_mode=pad_mode, power=power, layout="btm").cpu().numpy()
    src = of.normalize(raw) if norm else raw.astype(np.float64)
    if pad_mode == "end":
        ref = of.raw_to_mel(src, plan.weights, 4096, 281, power=power)
    else:
        ref = of.get_spect(src, plan.weights, 4096, 281, power, pad_mode)
    _rel_close(out, ref.transpose(0, 2, 1), 2e-5)


def test_mel_short_and_empty(fe, cuda):
    plan = _plan(fe)
    raw = synth_clips(2, n=5000, seed=10)
    x = torch.from_numpy(raw).to(cuda)
    out = plan.mel(x, fe.normalize_stats(x)).cpu().numpy()
    ref = of.raw_to_mel(of.normalize(raw), plan.weights).transpose(0, 2, 1)
    assert out.shape[1] == -(-5000 // 281)
    _rel_close(out, ref, 2e-5)
    e = plan.mel(torch.zeros((0, 144000), device=cuda))
    assert e.shape == (0, 513, 128)


def _mel_batch(fe, cuda, b, seed):
    raw = synth_clips(b, seed=seed)
    plan = _plan(fe)
    x = torch.from_numpy(raw).to(cuda)
    return plan.mel(x, fe.normalize_stats(x), layout="btm")


def test_pcen_forward(fe, cuda):
    mel = _mel_batch(fe, cuda, 2, 12)
    p = torch.tensor([0.98, 2.0, 2.0, 0.04], device=cuda)
    out = fe.pcen(mel, p).cpu().numpy()
    ref = of.pcen(mel.cpu().numpy().astype(np.float64)).transpose(0, 2, 1)
    assert out.shape == (2, 128, 513)
    assert np.abs(out - ref).max() <= 5e-5
    assert out.min() == -1.0 and out.max() == 1.0
    ob = fe.pcen(mel, p, out_dtype=torch.bfloat16).float().cpu().numpy()
    assert np.abs(ob - ref).max() <= 8e-3


@pytest.mark.parametrize("params", [(0.98, 2.0, 2.0, 0.04), (0.5, 1.5, 3.0, 0.2)])
def test_pcen_backward(fe, cuda, params):
    from oracle.torch_ref import pcen_torch

    mel = _mel_batch(fe, cuda, 2, 13)
    g = torch.randn((2, 128, 513), generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    p = torch.tensor(params, device=cuda, requires_grad=True)
    out = fe.pcen(mel, p)
    (out * g.float().to(cuda)).sum().backward()
    pr = torch.tensor(params, dtype=torch.float64, requires_grad=True)
    ref = pcen_torch(mel.cpu().double(), pr)
    (ref * g).sum().backward()
    gg, gr = p.grad.cpu().double().numpy(), pr.grad.numpy()
    np.testing.assert_allclose(gg, gr, rtol=2e-3, atol=2e-3 * np.abs(gr).max())


@pytest.mark.parametrize("power", [1, 2])
def test_mel_from_spec_golden(fe, cuda, power):
    """acfe_mel_from_spec (the load_raw=False path, tfdataset.py:1082-1090) on the
    golden |S| fixtures against the reference custommel.mel_spec output
    (tests/golden/mel_spec_p{1,2}.npz, generated from the reference itself):
    three clips at a clip stride, both output layouts; the plan's own
    filterbank is pinned separately (bit-exact mel_f goldens)."""
    import numpy as np
    from conftest import GOLDEN

    d = np.load(GOLDEN / f"mel_spec_p{power}.npz")
    S, ref = d["S"].astype(np.float32), d["mel"].astype(np.float64)   # [2049, T], [128, T]
    T = S.shape[1]
    plan = fe.MelPlan(n_mels=128)
    spec = torch.from_numpy(np.stack([S, 0.5 * S, S[:, ::-1].copy()])).to(cuda)
    refs = [ref, 0.5 ** power * ref, None]
    for layout in ("btm", "bmt"):
        out = plan.mel_from_spec(spec, power=power, layout=layout).double().cpu().numpy()
        if layout == "btm":
            out = out.transpose(0, 2, 1)
        for b, r in enumerate(refs):
            if r is None:  # time-reversed clip: same weights, reversed frames
                r = out[0][:, ::-1] * 1.0
                assert np.allclose(out[b], r, rtol=1e-6, atol=1e-6 * np.abs(r).max())
                continue
            assert np.abs(out[b] - r).max() <= 2e-6 * np.abs(r).max(), (b, layout)


def test_stored_spectrogram_path_matches_raw_path(fe, cuda):
    """The stored spectrogram of build.py (|centre-padded STFT| of the
    normalised clip, audiodataset.py:1302-1303) through acfe_mel_from_spec
    equals the fused raw-audio kernel run with the same framing
    (acfe_mel_fwd, centre / constant padding, power 1), and the full
    FrontEnd.forward_spec (PCEN) equals PCEN of the oracle mel."""
    import numpy as np
    import build
    from acfe.train import FrontEnd
    from oracle import frontend as of

    rng = np.random.default_rng(9)
    clips = np.stack([build.synth_clip(rng, i == 1) for i in range(3)])
    spec = torch.from_numpy(np.stack([build.stft_magnitude(c) for c in clips])).to(cuda)
    plan = fe.MelPlan(n_mels=128)
    a = plan.mel_from_spec(spec, power=1, layout="btm")
    x = torch.from_numpy(clips).to(cuda)
    b = plan.mel(x, fe.normalize_stats(x), pad_mode="constant", power=1, layout="btm")
    rel = ((a - b).norm() / b.norm()).item()
    assert rel < 1e-5, rel
    front = FrontEnd(n_mels=128, dtype=torch.float32, device=cuda).to(cuda)
    got = front.forward_spec(spec).detach().double().cpu().numpy()
    mel = np.einsum("mf,bft->btm", plan.weights.astype(np.float64), spec.double().cpu().numpy())
    ref = of.pcen(mel).transpose(0, 2, 1)
    assert np.abs(got - ref).max() < 5e-5


def test_normalize_reference_golden_bitexact(fe, cuda):
    """Row a1 pinned to the reference itself (tests/golden/normalize_golden.npz,
    made by oracle/gen_golden_normalize.py from predict_utils.normalize_data /
    audiodataset.normalize_data, float32): acfe_normalize_stats +
    acfe_normalize_apply bit for bit on every clip (3 s clips batched as
    tfdataset.normalize sees them, a 5 000-sample clip, a lone spike, a
    constant clip whose 0 / 0 is NaN) and on the load_samples(normalize=True)
    windows (zero-padded short tracks: the pads take part in the min / max).
    The fused users of the same arithmetic: acfe_mixup (normalize-on-load of
    both inputs, tfdataset.py:950 blend) bit for bit against the float32
    oracle composition that the fixture pins, and acfe_mel_fwd's
    normalize-on-load (Markstein reciprocal division, frontend.hip norm1r) ==
    mel of the separately normalised clips, bit for bit."""
    from oracle.gen_golden_normalize import N, SR, STRIDE, clip_set, hash_audio, sha

    z = np.load(GOLDEN / "normalize_golden.npz")
    clips = clip_set()
    full = np.stack([clips["full0"], clips["full1"], clips["full2"]])
    y = fe.normalize(torch.from_numpy(full).to(cuda)).cpu().numpy()
    for r, name in enumerate(("full0", "full1", "full2")):
        assert np.array_equal(y[r, ::STRIDE], z[f"norm_{name}_sample"]), name
        assert sha(y[r]) == str(z[f"norm_{name}_sha"]), name
    for name in ("short", "spike", "const"):
        yy = fe.normalize(torch.from_numpy(clips[name][None]).to(cuda)).cpu().numpy()[0]
        if f"norm_{name}_sha" in z:
            assert sha(yy) == str(z[f"norm_{name}_sha"]), name
        else:
            assert np.array_equal(yy, z[f"norm_{name}"], equal_nan=True), name

    recs = {}
    wins = []
    for k, ti, first, src, cnt in z["ls_rows"]:
        rec = recs.setdefault(int(k), hash_audio(SR * 20, 100 + int(k), 0.8))
        w = np.zeros(N, np.float32)
        w[first:first + cnt] = rec[src:src + cnt]
        wins.append(w)
    yw = fe.normalize(torch.from_numpy(np.stack(wins)).to(cuda)).cpu().numpy()
    for r in range(len(wins)):
        assert sha(yw[r]) == str(z["ls_sha"][r]), r

    # mix_up with both normalizations on load, then the second normalize
    x1 = torch.from_numpy(full).to(cuda)
    x2 = torch.from_numpy(full[::-1].copy()).to(cuda)
    lam = torch.tensor([0.3, 1.0, 0.0], device=cuda)
    mixed = fe.mix_up(x1, x2, lam, fe.normalize_stats(x1), fe.normalize_stats(x2))
    ref = of.mix_up_f32(of.normalize_f32(full), of.normalize_f32(full[::-1]), lam.cpu().numpy())
    assert np.array_equal(mixed.cpu().numpy(), ref)
    assert np.array_equal(fe.normalize(mixed).cpu().numpy(), of.normalize_f32(ref))

    # the mel kernel's normalize-on-load == mel of the normalised clips
    plan = fe.MelPlan(n_mels=128)
    a = plan.mel(x1, fe.normalize_stats(x1))
    b = plan.mel(fe.normalize(x1), None)
    assert torch.equal(a, b)


@pytest.mark.parametrize("fpw", [1, 3, 4, 8])
@pytest.mark.parametrize("n_mels,pad_mode,norm,power,n", [(128, "end", True, 2, 144000), (160, "constant", True, 2, 144000),
                                                          (128, "reflect", False, 1, 144000), (40, "end", True, 2, 144000),
                                                          (128, "end", False, 2, 5000), (96, "constant", False, 1, 9000)])
def test_mel_one_wave_per_frame(fe, cuda, fpw, n_mels, pad_mode, norm, power, n):
    """k_mel_w5 (one wave per frame, acfe_mel_w5_frames(f)) is bit-identical to
    k_mel_w4 -- same arithmetic per value, only the thread mapping and the
    synchronisation differ -- across framings, normalise-on-load, power 1 / 2,
    a 40-mel 1.5 kHz plan, short clips and frame counts that leave the last
    wave's walk partial; and within the 2e-5 bound of the float64 oracle."""
    from acfe._lib import lib

    raw = synth_clips(3, n=n, seed=23)
    plan = _plan(fe, n_mels=n_mels, fmax=11000 if n_mels != 40 else 1500)
    x = torch.from_numpy(raw).to(cuda)
    st = fe.normalize_stats(x) if norm else None
    prev = lib.acfe_mel_w5_frames(0)
    try:
        ref4 = plan.mel(x, st, pad_mode=pad_mode, power=power, layout="btm").cpu().numpy()
        lib.acfe_mel_w5_frames(fpw)
        out5 = plan.mel(x, st, pad_mode=pad_mode, power=power, layout="btm").cpu().numpy()
        out5t = plan.mel(x, st, pad_mode=pad_mode, power=power, layout="bmt").cpu().numpy()
    finally:
        lib.acfe_mel_w5_frames(prev)
    np.testing.assert_array_equal(out5, ref4)
    np.testing.assert_array_equal(out5t, out5.transpose(0, 2, 1))
    src = of.normalize(raw) if norm else raw.astype(np.float64)
    if pad_mode == "end":
        ref = of.raw_to_mel(src, plan.weights, 4096, 281, power=power)
    else:
        ref = of.get_spect(src, plan.weights, 4096, 281, power, pad_mode)
    _rel_close(out5, ref.transpose(0, 2, 1), 2e-5)
