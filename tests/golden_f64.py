"""Helpers for the float64 fixtures (tests/golden/codec_f64.npz, gen_golden.py ``f64``): case inputs, bit
comparison of float64 vectors, the oracle call of each case name and the tie-tolerant top-k rule on float64 keys."""

from __future__ import annotations

import random
from typing import Dict, Tuple

import numpy as np

from oracle import compressors_ref as ref
from tests import golden_cases as gc


def load() -> Dict[str, Dict[str, np.ndarray]]:
    return gc.load("codec_f64.npz")


def make_input64(D: int, seed: int, zero_frac: float = 0.05, scale: float = 1e-3) -> np.ndarray:
    """Same recipe as gen_golden.make_input64."""
    g = np.random.default_rng(30_000 + seed * 7919 + D)
    x = g.standard_normal(D) * scale
    if D > 1:
        x[g.random(D) < zero_frac] = 0.0
    return x


def case_input(case: str, rec: Dict[str, np.ndarray]) -> np.ndarray:
    if "x" in rec:
        return rec["x"]
    parts = case.split("|")
    D, seed = int(parts[1]), int(parts[-1])
    if parts[0] == "adaptive_heavy":  # Cauchy, 20 % zeros (gen_golden.gen_f64)
        g = np.random.default_rng(40_000 + seed * 104729 + D)
        x = g.standard_cauchy(D) * 1e-3
        x[g.random(D) < 0.2] = 0.0
    else:
        x = make_input64(D, seed)
    assert gc.sha(x) == str(rec["sha_x"]), f"input recipe drifted for {case}"
    return x


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    """Bit-identical float64 vectors, except that any NaN equals any NaN."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    an, bn = np.isnan(a), np.isnan(b)
    return bool(np.array_equal(an, bn) and np.array_equal(a.view(np.uint64)[~an], b.view(np.uint64)[~bn]))


def check_output(rec: Dict[str, np.ndarray], out: np.ndarray) -> bool:
    if "out" in rec:
        return same_bits(out, rec["out"])
    return gc.sha(out) == str(rec["sha_out"])


def dense_params(name: str) -> Tuple[str, int, float, bool]:
    """(kind, levels, p, fp64_stats) of a dithering case name."""
    if name.startswith("std64_L"):
        L, pn = name[len("std64_L"):].split("_")
        return "std", int(L), (np.inf if pn == "inf" else 2), True
    kind = "std" if name.startswith("std") else "nat"
    fp64 = "64" in name.split("_")[0]
    L = int(name.split("_")[1][1:])
    p = np.inf if name.endswith("inf") else 2
    return kind, L, p, fp64


def oracle_dense(name: str, x: np.ndarray):
    stream = ref.python_random_stream()
    if name == "identical":
        return ref.identical(x)
    if name.startswith("lazy"):
        return ref.lazy(x, 0.3 if name == "lazy_p03" else 0.9, random.random())
    if name in ("natural32", "natural64"):
        out, send, _ = ref.natural(x, stream, fp64_stats=(name == "natural64"))
        return out, send
    kind, L, p, fp64 = dense_params(name)
    fn = ref.standard_dithering if kind == "std" else ref.natural_dithering
    out, send, _ = fn(x, L, p, stream, fp64_stats=fp64)
    return out, send


def order_keys64(x: np.ndarray) -> np.ndarray:
    """np.argsort order as uint64 keys: -0 == +0, NaN largest (the device's order_key64)."""
    b = np.ascontiguousarray(x, dtype=np.float64).view(np.uint64).copy()
    sign = np.uint64(1 << 63)
    b[b == sign] = 0
    k = np.where(b & sign, ~b, b | sign).astype(np.uint64)
    k[np.isnan(x)] = np.uint64(0xFFFFFFFFFFFFFFFF)
    return k


def topk_valid(x: np.ndarray, out: np.ndarray, K: int) -> bool:
    """gc.topk_valid on float64 keys: above the K-th largest kept bit for bit, below +0, K - #above ties kept."""
    if K <= 0 or K >= len(x):
        return same_bits(out, x)
    keys = order_keys64(x)
    t = np.sort(keys)[len(x) - K]
    above, below, tie = keys > t, keys < t, keys == t
    if not same_bits(out[above], x[above]):
        return False
    if np.any(out[below].view(np.uint64) != 0):
        return False
    xb, ob = x.view(np.uint64), out.view(np.uint64)
    kept = (ob[tie] == xb[tie]) | (np.isnan(out[tie]) & np.isnan(x[tie]))
    if not np.all(kept | (ob[tie] == 0)):
        return False
    if x[tie][0] == 0:
        return True
    return int(kept.sum()) == K - int(above.sum())
