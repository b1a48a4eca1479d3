"""Keras weight files <-> the acfe WRResNet modules.

The reference saves `{run}.keras` (model.save, audiomodel.py:515-518: a zip
holding `model.weights.h5`) and `*.weights.h5` checkpoints
(ModelCheckpoint(save_weights_only=True), audiomodel.py:878-938), and
predict.py loads them (predict.py:746-789).  Keras 3 lays a weights file out
as `layers/<layer name>/vars/<i>`, the variables of a layer in
`trainable + non_trainable` order:
  Conv2D              0 kernel [R, S, Cin, K] (RSCK), 1 bias [K]
  BatchNormalization  0 gamma, 1 beta, 2 moving_mean, 3 moving_variance
  Dense               0 kernel [in, out], 1 bias [out]
The acfe modules keep the reference layer names where the reference sets one
(conv1_1, res{s}{b}_branch*, bn{s}{b}_branch*, final_bn, prediction); the
layers the reference leaves unnamed (wr_resnet_bird's stem BN, shortcut and
head convolutions and head BNs; wr_resnet's shortcut convolutions) get Keras
auto-names (`conv2d`, `conv2d_1`, ... in creation order, offset by whatever
the session created before), so they are matched by class and creation
order: the file's auto-named layers of a class sorted by their numeric
suffix <-> the module's unnamed layers of that class in construction order.
Conv kernels are stored KRSC here (w_keras = w.permute(1, 2, 3, 0)).

Parity is unpinned: the reference ships no checkpoint and h5py is absent, so
the reader is exercised on files this module's writer produces in the Keras 3
layout (tests/test_keras_weights.py).
"""
from __future__ import annotations

import io
import re
import zipfile
from pathlib import Path

import numpy as np
import torch

import h5lite

_AUTO = re.compile(r"^(conv2d|batch_normalization|dense)(?:_(\d+))?$")


def _kind(mod) -> str | None:
    cls = type(mod).__name__
    if cls in ("Conv2D", "StemConv2D"):
        return "conv2d"
    if cls == "BatchNormalization":
        return "batch_normalization"
    if cls == "Dense":
        return "dense"
    return None


def keras_layers(model: torch.nn.Module):
    """[(keras class, reference layer name or None if auto-named, module)] in
    construction (= Keras creation) order."""
    out = []
    for mod in model.modules():
        k = _kind(mod)
        if k is not None:
            out.append((k, None if getattr(mod, "keras_auto", False) else mod.name, mod))
    return out


def _vars(kind, mod):
    """The module's tensors in Keras variable order, with their Keras layout
    converters (torch -> keras, keras -> torch)."""
    if kind == "conv2d":
        return [(mod.weight, lambda t: t.permute(1, 2, 3, 0), lambda a: a.permute(3, 0, 1, 2)),
                (mod.bias, None, None)]
    if kind == "batch_normalization":
        return [(mod.gamma, None, None), (mod.beta, None, None), (mod.moving_mean, None, None),
                (mod.moving_variance, None, None)]
    return [(mod.kernel, None, None), (mod.bias, None, None)]


def _read(path) -> dict:
    p = Path(path)
    data = p.read_bytes()
    if data[:2] == b"PK":  # .keras zip archive
        with zipfile.ZipFile(io.BytesIO(data)) as z:
            name = next((n for n in z.namelist() if n.endswith(".weights.h5")), None)
            if name is None:
                raise ValueError(f"{path}: no *.weights.h5 member in the .keras archive")
            data = z.read(name)
    flat = h5lite.read_h5(data)
    layers: dict[str, dict[int, np.ndarray]] = {}
    for key, arr in flat.items():
        parts = key.split("/")
        if len(parts) >= 3 and parts[-2] == "vars" and parts[-1].isdigit():
            layers.setdefault(parts[-3], {})[int(parts[-1])] = arr
    return {k: [v[i] for i in sorted(v)] for k, v in layers.items()}


def load_keras_weights(model: torch.nn.Module, path, strict=True) -> dict:
    """Load a Keras `.weights.h5` / `.keras` file into `model` (an acfe
    WRResNet); returns {"loaded": n_layers, "skipped": [...]}."""
    file_layers = _read(path)
    mine = keras_layers(model)
    named = {name for _, name, _ in mine if name is not None}
    # auto-named file layers per class, in creation order
    auto: dict[str, list[str]] = {}
    for name in file_layers:
        m = _AUTO.match(name)
        if m and name not in named:
            auto.setdefault(m.group(1), []).append(name)
    for k in auto:
        auto[k].sort(key=lambda n: int(_AUTO.match(n).group(2) or 0))
    want_auto: dict[str, int] = {}
    for kind, name, _ in mine:
        if name is None:
            want_auto[kind] = want_auto.get(kind, 0) + 1
    for kind, n in want_auto.items():
        if len(auto.get(kind, [])) != n:
            raise ValueError(f"{path}: {len(auto.get(kind, []))} auto-named {kind} layers in the file, the model has {n}")
    taken = {k: 0 for k in auto}
    loaded, used = 0, set()
    with torch.no_grad():
        for kind, name, mod in mine:
            if name is None:
                fname = auto[kind][taken[kind]]
                taken[kind] += 1
            else:
                fname = name
            if fname not in file_layers:
                if strict:
                    raise KeyError(f"{path}: layer {fname!r} not in the file")
                continue
            arrs = file_layers[fname]
            spec = _vars(kind, mod)
            if len(arrs) != len(spec):
                raise ValueError(f"{fname}: {len(arrs)} variables in the file, {len(spec)} expected")
            for (t, _, to_torch), a in zip(spec, arrs):
                v = torch.from_numpy(np.ascontiguousarray(a)).to(torch.float32)
                if to_torch is not None:
                    v = to_torch(v)
                if tuple(v.shape) != tuple(t.shape):
                    raise ValueError(f"{fname}: shape {tuple(v.shape)} vs model {tuple(t.shape)}")
                t.copy_(v.to(t.device))
            used.add(fname)
            loaded += 1
    skipped = sorted(set(file_layers) - used)
    return {"loaded": loaded, "skipped": skipped}


def keras_weights_tree(model: torch.nn.Module, auto_offset: dict | None = None) -> dict:
    """The model's weights as the Keras 3 weights-file tree {layers: {name: {vars: {i: array}}}}."""
    counters = dict(auto_offset or {})
    layers = {}
    for kind, name, mod in keras_layers(model):
        if name is None:
            i = counters.get(kind, 0)
            counters[kind] = i + 1
            name = kind if i == 0 else f"{kind}_{i}"
        vs = {}
        for j, (t, to_keras, _) in enumerate(_vars(kind, mod)):
            v = t.detach().float().cpu()
            if to_keras is not None:
                v = to_keras(v)
            vs[str(j)] = v.contiguous().numpy()
        layers[name] = {"vars": vs}
    return {"layers": layers, "vars": {}}


def save_keras_weights(model: torch.nn.Module, path, auto_offset: dict | None = None) -> Path:
    """Write `model` as a Keras 3 `*.weights.h5` (what the reference's
    ModelCheckpoint(save_weights_only=True) produces)."""
    p = Path(path)
    p.write_bytes(h5lite.write_h5(keras_weights_tree(model, auto_offset)))
    return p
