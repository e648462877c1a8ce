"""ORACLE — test infrastructure only.  Never imported by the product package (fl_sim_amd/).

A vectorised numpy restatement of the reference codec, ``fl_sim/compressors/compressors.py``
(wenh06/fl-sim), used by ``tests/`` as the parity checker for the HIP kernels, by
``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline`` leg.  Pinned against the
reference itself: ``tests/golden/*.npz`` were produced by running the reference's own
``Compressor.compressVector`` (``tests/golden/gen_golden.py``) and ``tests/test_oracle_golden.py``
checks this module reproduces them bit for bit.

RNG: every stochastic function takes the uniforms it consumes explicitly — either the compat stream
(what ``random.random()`` yields, in index order of the consuming elements) or the device's Philox
stream (``philox_uniforms``, one uniform per element index) — so the same function checks both
kernel modes.
"""

from __future__ import annotations

import math
from typing import Callable, Optional, Tuple

import numpy as np

F32 = np.float32
F64 = np.float64


# ------------------------------------------------------------------------------------------- levels
def standard_levels(s: int) -> np.ndarray:
    """compressors.py:157/172 ``np.arange(0, 1.1, 1/s)``: lv[i] = i * (1/s); lv[s] pinned to 1."""
    step = 1.0 / s
    lv = np.arange(s + 1, dtype=F64) * step
    lv[-1] = 1.0
    return lv


def natural_levels(s: int) -> np.ndarray:
    """compressors.py:194-197: [0, 2^-(s-1), ..., 1/2, 1]."""
    lv = np.zeros(s + 1, dtype=F64)
    lv[1:] = np.ldexp(1.0, np.arange(1, s + 1) - s)
    return lv


# ---------------------------------------------------------------------------------------------- philox
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al. 2011) on uint32 arrays; same round structure as flc_device.hpp."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32).copy() for v in (c0, c1, c2, c3))
    k0 = np.full_like(c0, k0, dtype=np.uint32)
    k1 = np.full_like(c0, k1, dtype=np.uint32)
    for _ in range(10):
        p0 = _M0 * c0.astype(np.uint64)
        p1 = _M1 * c2.astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = k0 + _W0
        k1 = k1 + _W1
    return c0, c1, c2, c3


def philox_uniforms(n: int, seed: int, counter: int, start: int = 0) -> np.ndarray:
    """u[e] for element indices e in [start, start + n): word (e & 3) of Philox group e >> 2, times 2^-32."""
    e = np.arange(start, start + n, dtype=np.uint64)
    g = e >> np.uint64(2)
    words = philox4x32_10(
        (g & np.uint64(0xFFFFFFFF)).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32),
        np.uint32(counter & 0xFFFFFFFF), np.uint32((counter >> 32) & 0xFFFFFFFF),
        np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF),
    )
    w = np.stack(words, axis=1)[np.arange(n), (e & np.uint64(3)).astype(np.int64)]
    return w.astype(F64) * 2.0**-32


def philox_uniforms_at(idx: np.ndarray, seed: int, counter: int) -> np.ndarray:
    """u[e] for the given element indices only (same stream as philox_uniforms)."""
    e = np.asarray(idx, dtype=np.uint64)
    g = e >> np.uint64(2)
    words = philox4x32_10(
        (g & np.uint64(0xFFFFFFFF)).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32),
        np.uint32(counter & 0xFFFFFFFF), np.uint32((counter >> 32) & 0xFFFFFFFF),
        np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF),
    )
    w = np.stack(words, axis=1)[np.arange(len(e)), (e & np.uint64(3)).astype(np.int64)]
    return w.astype(F64) * 2.0**-32


# ------------------------------------------------------------------------------------------ compressors
def identical(x: np.ndarray):
    """compressors.py:273-275."""
    return +x, x.shape[0]


def lazy(x: np.ndarray, P: float, testp: float):
    """compressors.py:276-283 (testp = the one random.random() drawn)."""
    if testp < P:
        return x / P, x.shape[0]
    return np.zeros_like(x), 0


def randk(x: np.ndarray, K: int, D: int, S: np.ndarray):
    """compressors.py:284-292 with S = the first K entries of the shuffled arange(D)."""
    out = np.zeros_like(x)
    out[S] = x.dtype.type(D / K) * x[S]  # a Python float times an element: x's dtype (fp32 rounds D / K first)
    return out, K


def topk_kept(x: np.ndarray, K: int) -> Tuple[np.ndarray, np.ndarray]:
    """Kept set of compressors.py:293-296 under a stable argsort: (ascending idx, values)."""
    order = np.argsort(x, kind="stable")
    kept = np.sort(order[len(x) - K:]) if 0 < K < len(x) else np.arange(len(x))
    return kept.astype(np.int64), x[kept]


def order_keys(x: np.ndarray) -> np.ndarray:
    """np.argsort order as uint32 keys: -0 == +0, NaN largest."""
    b = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).copy()
    b[b == 0x80000000] = 0
    k = np.where(b & np.uint32(0x80000000), ~b, b | np.uint32(0x80000000)).astype(np.uint32)
    k[np.isnan(x)] = 0xFFFFFFFF
    return k


def topk_kept_select(x: np.ndarray, K: int) -> Tuple[np.ndarray, np.ndarray]:
    """topk_kept in O(n) (np.partition on order keys): every key above the K-th largest, then the
    highest-indexed ties — the same set a stable ascending argsort keeps."""
    n = len(x)
    if not 0 < K < n:
        return topk_kept(x, K)
    keys = order_keys(x)
    t = np.partition(keys, n - K)[n - K]
    above = np.flatnonzero(keys > t)
    ties = np.flatnonzero(keys == t)
    kept = np.sort(np.concatenate([above, ties[len(ties) - (K - len(above)):]]))
    return kept.astype(np.int64), x[kept]


def randk_philox_indices(D: int, K: int, seed: int, counter: int) -> np.ndarray:
    """The device's philox-mode rand-k set: the K largest of the keys (Philox word >> 2 as an fp32 bit pattern)."""
    if K >= D:
        return np.arange(D, dtype=np.int64)
    words = (philox_uniforms(D, seed, counter) * 2.0**32).astype(np.uint64).astype(np.uint32)
    keys = (words >> np.uint32(2)).view(np.float32)
    return topk_kept_select(keys, K)[0]


def topk(x: np.ndarray, K: int):
    """compressors.py:293-296, ties resolved as a stable ascending argsort (highest indices kept)."""
    out = x.copy()
    if K != 0:  # order[:-0] is empty: K == 0 keeps everything (verified quirk of the reference)
        order = np.argsort(out, kind="stable")
        out[order[:-K]] = 0
    return out, K


def topk_threshold(x: np.ndarray, K: int) -> float:
    """The K-th largest value (the tie class any valid kept set must straddle)."""
    return np.sort(x, kind="stable")[len(x) - K]


def natural(x: np.ndarray, u_of: Callable[[np.ndarray], np.ndarray], fp64_stats: bool = False):
    """compressors.py:302-325.  ``u_of(nz_idx)`` returns the uniforms of the nonzero elements
    (compat: the next len(nz_idx) random.random() values; philox: u by element index)."""
    if x.dtype == F64:
        return natural64(x, u_of, fp64_stats)
    d = x.shape[0]
    out = np.zeros_like(x)
    nz = np.nonzero(x != 0.0)[0]
    if len(nz):
        xi = x[nz]
        ax = np.abs(xi).astype(F64)
        m, e = np.frexp(ax)              # ax = m * 2^e, m in [0.5, 1)
        down = e - 1                      # floor(log2 |x|)
        up = np.where(m == 0.5, down, down + 1)
        pt = ((np.ldexp(1.0, up) - ax) / np.ldexp(1.0, down)).astype(F32)  # exact
        u = u_of(nz)
        expo = np.where(u < pt.astype(F64), down, up)
        out[nz] = (np.sign(xi) * np.ldexp(1.0, expo)).astype(x.dtype)
    send = 12.0 / 64.0 * d if fp64_stats else 9.0 / 32.0 * d
    return out, send, len(nz)


def natural64(x: np.ndarray, u_of: Callable[[np.ndarray], np.ndarray], fp64_stats: bool = False):
    """compressors.py:302-325 on a float64 vector: every step in fp64, ``math.log2`` / ``math.floor`` /
    ``math.ceil`` per element exactly as the reference evaluates them (a power of two gives down == up, pt = 0)."""
    d = x.shape[0]
    out = np.zeros_like(x)
    nz = np.nonzero(x != 0.0)[0]
    if len(nz):
        ax = np.abs(x[nz])
        alpha = [math.log2(a) for a in ax.tolist()]
        down = np.array([math.floor(a) for a in alpha], dtype=np.int64)
        up = np.array([math.ceil(a) for a in alpha], dtype=np.int64)
        pt = (np.ldexp(1.0, up) - ax) / np.ldexp(1.0, down)
        u = u_of(nz)
        out[nz] = np.sign(x[nz]) * np.ldexp(1.0, np.where(u < pt, down, up))
    send = 12.0 / 64.0 * d if fp64_stats else 9.0 / 32.0 * d
    return out, send, len(nz)


def vector_norm(x: np.ndarray, p: float):
    """np.linalg.norm(x, p) as the reference calls it (compressors.py:332, 372), in x's dtype."""
    return x.dtype.type(np.linalg.norm(x, p)) if x.dtype == F64 else F32(np.linalg.norm(x, p))


def dither64(x: np.ndarray, levels: np.ndarray, pnorm: np.float64, u_of: Callable[[np.ndarray], np.ndarray]):
    """compressors.py:339-357 / 376-394 on a float64 vector: y = |x| / norm, the level bracket, p and the decoded
    value lv * sign * norm all in fp64.  A y above 1 (a p = 2 norm that underflowed to 0) has no bracket: the
    reference's loop then indexes past the table, and so does this (IndexError)."""
    out = np.zeros_like(x)
    nz = np.nonzero(x != 0.0)[0]
    lvl_idx = np.zeros(len(x), dtype=np.int64)
    if len(nz) == 0:
        return out, 0, nz, lvl_idx
    xi = x[nz]
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        yi = np.abs(xi) / pnorm
    cons = ~np.isnan(yi)
    if np.any(yi[cons] > 1.0):
        raise IndexError(f"index {len(levels)} is out of bounds for axis 0 with size {len(levels)}")
    ci = nz[cons]
    lvl = np.zeros(len(nz), dtype=F64)
    if len(ci):
        y = yi[cons]
        j = np.searchsorted(levels, y, side="left")
        s = np.maximum(j - 1, 0)
        p = (y - levels[s + 1]) / (levels[s] - levels[s + 1])
        li = np.where(u_of(ci) < p, s, s + 1)
        lvl[cons] = levels[li]
        lvl_idx[ci] = li
    with np.errstate(invalid="ignore", over="ignore"):
        out[nz] = (lvl * np.sign(xi)) * pnorm
    return out, len(nz), ci, lvl_idx


def dither(x: np.ndarray, levels: np.ndarray, pnorm: np.float32, u_of: Callable[[np.ndarray], np.ndarray]):
    """Per-element rule of compressors.py:339-357 / 376-394 for a given level table and norm.
    Returns (out, nnz, consumer_idx, level_idx) — consumers are the elements that draw a uniform."""
    out = np.zeros_like(x)
    nz = np.nonzero(x != 0.0)[0]
    lvl_idx = np.zeros(len(x), dtype=np.int64)
    if len(nz) == 0:
        return out, 0, nz, lvl_idx
    xi = x[nz]
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        yi = (np.abs(xi) / pnorm).astype(F32)
    cons = ~np.isnan(yi)
    ci = nz[cons]
    lvl = np.zeros(len(nz), dtype=F64)
    if len(ci):
        y64 = yi[cons].astype(F64)
        j = np.searchsorted(levels, y64, side="left")
        s = np.maximum(j - 1, 0)
        p = (y64 - levels[s + 1]) / (levels[s] - levels[s + 1])
        u = u_of(ci)
        take_lo = u < p
        li = np.where(take_lo, s, s + 1)
        lvl[cons] = levels[li]
        lvl_idx[ci] = li
    with np.errstate(invalid="ignore", over="ignore"):
        out[nz] = (lvl.astype(F32) * np.sign(xi)) * pnorm
    return out, len(nz), ci, lvl_idx


def standard_dithering(x, s, p, u_of, pnorm=None, fp64_stats=False, norm_send=1):
    """compressors.py:327-365 (norm compressor = identical: it sends 1 component)."""
    if x.dtype == F64:
        pn = vector_norm(x, p) if pnorm is None else F64(pnorm)
        out, nnz, _, _ = dither64(x, standard_levels(s), pn, u_of)
    else:
        pn = vector_norm(x, p) if pnorm is None else F32(pnorm)
        out, nnz, _, _ = dither(x, standard_levels(s), pn, u_of)
    per = (1.0 + np.ceil(math.log2(s))) / (64.0 if fp64_stats else 32.0)
    send = norm_send
    for _ in range(nnz if nnz < 4096 else 0):
        send += per
    if nnz >= 4096:
        send = norm_send + nnz * per  # exact: multiples of 1/64 below 2^46
    return out, send, pn


def natural_dithering(x, s, p, u_of, pnorm=None, fp64_stats=False):
    """compressors.py:367-404."""
    if x.dtype == F64:
        pn = vector_norm(x, p) if pnorm is None else F64(pnorm)
        out, _, _, _ = dither64(x, natural_levels(s), pn, u_of)
    else:
        pn = vector_norm(x, p) if pnorm is None else F32(pnorm)
        out, _, _, _ = dither(x, natural_levels(s), pn, u_of)
    d = x.shape[0]
    send = d * (1.0 + np.ceil(math.log2(s))) / (64.0 if fp64_stats else 32.0)
    return out, send, pn


def stacked(x: np.ndarray, K: int, s: int, u_of: Callable[[np.ndarray], np.ndarray], fast: bool = False):
    """Top-K then standard dithering (p = inf) of the K-sparse result — the pipeline the fused
    flc_stacked_encode implements.  Returns (dense out, kept idx, codes (sign<<7 | level), norm).
    ``fast`` selects the kept set with topk_kept_select (same set, O(n))."""
    kept, vals = (topk_kept_select if fast else topk_kept)(x, K)
    y = np.zeros_like(x)
    y[kept] = vals
    pn = F32(np.max(np.abs(y))) if len(y) else F32(0)
    out, _, _, lvl_idx = dither(y, standard_levels(s), pn, u_of)
    codes = (lvl_idx[kept] | (np.signbit(vals).astype(np.int64) << 7)) * (vals != 0)
    return out, kept, codes.astype(np.uint8), pn


def adaptive_random(x: np.ndarray, D: int, u: float):
    """compressors.py:297-301 with u = the one random_sample() np.random.choice draws."""
    ax = np.abs(x)
    p = ax / ax.sum()
    cdf = p.astype(F64).cumsum()
    cdf /= cdf[-1]
    ind = int(cdf.searchsorted(u, side="right"))
    out = np.zeros_like(x)
    out[ind] = x[ind]
    return out, 1, ind


# ------------------------------------------------------------------------------------------------ rng
def compat_stream(draw: Callable[[int], np.ndarray]):
    """u_of for compat mode: consuming elements take the next uniforms of ``draw`` in index order."""

    def u_of(idx: np.ndarray) -> np.ndarray:
        return np.asarray(draw(len(idx)), dtype=F64)

    return u_of


def python_random_stream():
    import random

    return compat_stream(lambda n: np.array([random.random() for _ in range(n)], dtype=F64))


def philox_stream(seed: int, counter: int, n_total: int, row_offset: int = 0):
    """u_of for philox mode: uniform of element e (flat index e + row_offset)."""
    u_all = philox_uniforms(n_total, seed, counter) if n_total else np.zeros(0)

    def u_of(idx: np.ndarray) -> np.ndarray:
        return u_all[idx + row_offset]

    return u_of
