"""The C-ABI library loads and exports every symbol include/acfe.h declares
(no compute calls: this runs without a GPU)."""
import re

from conftest import ROOT


def header_functions():
    txt = (ROOT / "include" / "acfe.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(acfe_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_api():
    fns = header_functions()
    assert "acfe_mel_fwd" in fns and "acfe_pcen_bwd" in fns


def test_library_exports_every_declared_symbol():
    from acfe import _lib

    missing = [f for f in header_functions() if not hasattr(_lib.lib, f)]
    assert not missing, missing


def test_binding_covers_header():
    from acfe import _lib

    assert sorted(_lib.SIGNATURES) == header_functions()


def test_host_only_calls():
    from acfe import _lib

    assert _lib.lib.acfe_version() >= 100
    assert _lib.lib.acfe_pcen_partials(512, 128) == 1024  # 64 (b, m) rows per PCEN workgroup
    # invalid arguments are reported, not crashed on
    assert _lib.lib.acfe_mel_filterbank(0, 128, 100.0, 11000.0, 4096, 1000.0, None) == _lib.E_INVAL


def header_param_counts():
    txt = (ROOT / "include" / "acfe.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(acfe_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", txt):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_binding_arity_matches_header():
    from acfe import _lib

    counts = header_param_counts()
    bad = {k: (len(v), counts[k]) for k, v in _lib.SIGNATURES.items() if len(v) != counts[k]}
    assert not bad, bad
