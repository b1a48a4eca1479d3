"""tfpcen (reference tfpcen.py:1-110) for the acfe path: trainable PCEN with
batch-global normalize_minmax, running on the HIP kernels."""
from acfe.frontend import PCEN, pcen  # noqa: F401
