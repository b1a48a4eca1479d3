"""acfe -- MI355X-native audio-classification front end + engine.

Host side of the hot path: thin torch-tensor wrappers over the C ABI in
include/acfe.h (libacfe.so, gfx950 HIP kernels).  Importing this package
without the built library raises ImportError; there is no CPU fallback.
"""
from . import _lib  # noqa: F401  (fails loudly if libacfe.so is missing)
from ._lib import AcfeError, lib  # noqa: F401
