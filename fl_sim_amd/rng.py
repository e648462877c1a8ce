"""Compat-mode RNG: keep the interpreter's global MT19937 streams in lock-step with the reference.

The reference draws stochastic-rounding uniforms from Python's global ``random`` module
(``compressors.py:277, 316, 349, 386``) and the Rand-K permutation from numpy's global legacy
``RandomState`` (``compressors.py:285-287``); ``set_seed`` (``fl_sim/utils/misc.py:196-217``) seeds
both.  Here the state is exported, advanced by the C library exactly as the interpreter would advance
it (``flc_mt_random_doubles`` / ``flc_np_shuffle_prefix``), and written back, so a compressor call
consumes the same draws the reference would and leaves both streams where the reference would.
"""

from __future__ import annotations

import random
from ctypes import POINTER, c_double, c_int32, c_uint32

import numpy as np

from . import _lib


def _py_state():
    version, internal, gauss = random.getstate()
    mt = np.array(internal[:624], dtype=np.uint32)
    pos = c_int32(int(internal[624]))
    return version, mt, pos, gauss


def python_random_doubles(n: int) -> np.ndarray:
    """Exactly ``[random.random() for _ in range(n)]``, computed by the C library; advances ``random``."""
    if n <= 0:
        return np.zeros(0, dtype=np.float64)
    version, mt, pos, gauss = _py_state()
    out = np.empty(n, dtype=np.float64)
    _lib.call(
        "flc_mt_random_doubles",
        mt.ctypes.data_as(POINTER(c_uint32)),
        pos,
        out.ctypes.data_as(POINTER(c_double)),
        n,
    )
    random.setstate((version, tuple(int(v) for v in mt) + (int(pos.value),), gauss))
    return out


def numpy_shuffle_prefix(D: int, K: int) -> np.ndarray:
    """``S = np.arange(D); np.random.shuffle(S); S[:K]`` on numpy's global legacy RandomState."""
    name, key, pos, has_gauss, cached = np.random.get_state()
    if name != "MT19937":
        raise RuntimeError(f"unexpected numpy bit generator {name}")
    mt = np.array(key, dtype=np.uint32)
    p = c_int32(int(pos))
    kk = min(K, D)
    out = np.empty(max(kk, 1), dtype=np.int32)
    _lib.call(
        "flc_np_shuffle_prefix",
        mt.ctypes.data_as(POINTER(c_uint32)),
        p,
        D,
        K,
        out.ctypes.data_as(POINTER(c_int32)),
    )
    np.random.set_state((name, mt, int(p.value), has_gauss, cached))
    return out[:kk]


def numpy_random_sample() -> float:
    """``np.random.random_sample()`` on numpy's global legacy RandomState (the draw ``np.random.choice``
    makes, compressors.py:298), advancing that stream exactly as numpy would."""
    name, key, pos, has_gauss, cached = np.random.get_state()
    if name != "MT19937":
        raise RuntimeError(f"unexpected numpy bit generator {name}")
    mt = np.array(key, dtype=np.uint32)
    p = c_int32(int(pos))
    out = np.empty(1, dtype=np.float64)
    _lib.call("flc_mt_random_doubles", mt.ctypes.data_as(POINTER(c_uint32)), p,
              out.ctypes.data_as(POINTER(c_double)), 1)
    np.random.set_state((name, mt, int(p.value), has_gauss, cached))
    return float(out[0])


class PhiloxStream:
    """Counter-based stream of the device kernels (Philox4x32-10 keyed by ``seed``).

    Each codec call consumes one counter value, so repeated calls are independent and a call's
    output is a pure function of (seed, counter, input) — reproducible regardless of launch geometry.
    """

    def __init__(self, seed: int = 0, counter: int = 0):
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = int(counter)

    def next(self) -> tuple:
        c = self.counter
        self.counter += 1
        return self.seed, c & 0xFFFFFFFFFFFFFFFF
