"""Keras weight files (f3): the Keras 3 `layers/<name>/vars/<i>` layout of
`*.weights.h5` and `.keras` archives (audiomodel.py:515-518, :878-938;
predict.py:746-789) read into / written from the acfe WRResNet modules.

Parity unpinned: the reference ships no checkpoint and h5py is absent here,
so the HDF5 subset reader (h5lite) is exercised on files its writer produces;
the layer-name mapping (reference names + auto-named layers by class and
creation order, whatever the session's auto-name offset) and the RSCK <-> KRSC
kernel transposition are checked by round trips between two differently
initialised models."""
import io
import zipfile

import numpy as np
import pytest
import torch


def _models(kind, classes=7):
    if kind == "bird":
        from resnet.wr_resnet_bird import WRResNet
    else:
        from resnet.wr_resnet import WRResNet
    a = WRResNet(input_shape=(128, 64, 3), classes=classes, seed=0)
    b = WRResNet(input_shape=(128, 64, 3), classes=classes, seed=5)
    with torch.no_grad():
        g = torch.Generator().manual_seed(1)
        for n, t in list(a.named_parameters()) + list(a.named_buffers()):
            t.copy_(torch.randn(t.shape, generator=g))
    return a, b


@pytest.mark.parametrize("kind", ["bird", "wrn"])
@pytest.mark.parametrize("offset", [None, {"conv2d": 6, "batch_normalization": 3}], ids=["fresh", "offset"])
def test_weights_h5_round_trip(tmp_path, kind, offset):
    from keras_weights import load_keras_weights, save_keras_weights

    a, b = _models(kind)
    f = save_keras_weights(a, tmp_path / "val_loss.weights.h5", auto_offset=offset)
    assert f.read_bytes()[:8] == b"\x89HDF\r\n\x1a\n"
    rep = load_keras_weights(b, f)
    assert rep["skipped"] == []
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_keras_layout_and_archive(tmp_path):
    """The file holds Keras's names and layouts: conv kernels RSCK, BN in
    gamma/beta/moving_mean/moving_variance order, the reference's names for
    named layers and conv2d / batch_normalization auto-names for the rest;
    a `.keras` zip with the weights member loads the same."""
    import h5lite
    from keras_weights import load_keras_weights, save_keras_weights

    a, b = _models("bird")
    f = save_keras_weights(a, tmp_path / "m.weights.h5")
    flat = h5lite.read_h5(f)
    w = a.blocks[0].conv21.weight.detach()
    assert np.array_equal(flat["layers/res1b0_branch21/vars/0"], w.permute(1, 2, 3, 0).numpy())
    assert np.array_equal(flat["layers/final_bn/vars/3"], a.final_bn.moving_variance.numpy())
    assert np.array_equal(flat["layers/batch_normalization/vars/0"], a.bn_stem.gamma.detach().numpy())
    # head (4, 10) conv: the 4th auto-named Conv2D after the three shortcuts
    assert flat["layers/conv2d_3/vars/0"].shape == (4, 10, 256, 128)
    assert flat["layers/prediction/vars/0"].shape == tuple(a.prediction.kernel.shape)
    z = tmp_path / "run.keras"
    with zipfile.ZipFile(z, "w") as zf:
        zf.writestr("config.json", "{}")
        zf.writestr("model.weights.h5", f.read_bytes())
    load_keras_weights(b, z)
    assert torch.equal(a.head_conv1.weight, b.head_conv1.weight)


def test_mismatch_is_an_error(tmp_path):
    from keras_weights import load_keras_weights, save_keras_weights

    a, _ = _models("bird", classes=7)
    _, c = _models("bird", classes=9)
    f = save_keras_weights(a, tmp_path / "x.weights.h5")
    with pytest.raises(ValueError):
        load_keras_weights(c, f)
