"""fl_sim_amd — MI355X-native gradient codec + aggregation path for fl-sim.

The hot path of wenh06/fl-sim's client->server update step, rebuilt for gfx950:

* :class:`Compressor` / :class:`CompressorType` — drop-in for ``fl_sim.compressors`` (compressors.py);
* :mod:`fl_sim_amd.aggregation` — ``add_parameters`` / ``avg_parameters`` / ``update_gradients`` /
  ``fedopt_update`` (nodes.py:1116-1180, _fedopt.py:196-265) and server mixins;
* :mod:`fl_sim_amd.dist` — one client shard per GPU, RCCL reduce of the decoded weighted deltas;
* :mod:`fl_sim_amd.codec` — the device-level functional API (wire packets, fused decode-accumulate);
* ``torch.ops.flcodec.*`` — the same entry points registered with the PyTorch dispatcher
  (``libflcodec_torch.so``, see :func:`load_torch_ops`).

All compute runs in ``libflcodec.so`` (hand-written HIP kernels, C ABI in ``include/flcodec.h``);
there is no CPU fallback.
"""

import os

from . import _lib
from .compressors import Compressor, CompressorType

__all__ = ["Compressor", "CompressorType", "native_library", "load_torch_ops", "__version__"]
__version__ = "0.1.0"


def native_library() -> str:
    """Load the HIP library (raises if missing) and return its path."""
    _lib.load()
    return _lib.LIB_PATH


TORCH_OPS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libflcodec_torch.so")


def load_torch_ops() -> str:
    """Register ``torch.ops.flcodec.*`` (HIP kernels plus Meta shape functions) and return the library path.

    Raises ImportError if ``libflcodec_torch.so`` was not built (``make -C fl_sim_amd/csrc torch``)."""
    import torch

    if not os.path.exists(TORCH_OPS_PATH):
        raise ImportError(f"{TORCH_OPS_PATH} not found: build it with `make -C fl_sim_amd/csrc torch`")
    if not hasattr(torch.ops.flcodec, "stacked_encode"):
        torch.ops.load_library(TORCH_OPS_PATH)
    return TORCH_OPS_PATH
