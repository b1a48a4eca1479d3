"""acfe -- MI355X-native audio-classification front end + engine.

Host side of the hot path: thin torch-tensor wrappers over the C ABI in
include/acfe.h (libacfe.so, gfx950 HIP kernels).  Every compute module
(frontend, ops, layers, train) imports `_lib`, which raises ImportError when
the built library is missing: there is no CPU fallback.  `acfe.dp` (the
torch.distributed plumbing) is HIP-free so the gloo tests import it alone.
"""


def __getattr__(name):
    if name in ("lib", "AcfeError"):
        from . import _lib

        return getattr(_lib, name)
    raise AttributeError(name)
