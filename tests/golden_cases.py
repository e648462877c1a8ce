"""Shared helpers: read the reference fixtures in tests/golden/ and map case names to oracle calls.

Case names are the ones gen_golden.py writes (``name|D|seed`` for dense codecs, ``name|D|K|seed``
for sparse ones, ``...|special:<vector>|...`` for hand-made edge vectors).
"""

from __future__ import annotations

import hashlib
import os
import random
from collections import defaultdict
from typing import Dict, Tuple

import numpy as np

from oracle import compressors_ref as ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def make_input(D: int, seed: int, zero_frac: float = 0.05, scale: float = 1e-3) -> np.ndarray:
    """Same recipe as gen_golden.make_input (does not touch the global streams)."""
    g = np.random.default_rng(10_000 + seed * 7919 + D)
    x = (g.standard_normal(D) * scale).astype(np.float32)
    if D > 1:
        x[g.random(D) < zero_frac] = 0.0
    return x


def load(name: str) -> Dict[str, Dict[str, np.ndarray]]:
    """{case_key: {field: array}} of one fixture file."""
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    cases: Dict[str, Dict[str, np.ndarray]] = defaultdict(dict)
    for k in z.files:
        case, field = k.rsplit("|", 1)
        cases[case][field] = z[k]
    return dict(cases)


def case_input(case: str, rec: Dict[str, np.ndarray]) -> np.ndarray:
    if "x" in rec:
        return rec["x"]
    parts = case.split("|")
    D, seed = int(parts[1]), int(parts[-1])
    x = make_input(D, seed, zero_frac=0.0 if parts[0] == "adaptive" else 0.05)
    assert sha(x) == str(rec["sha_x"]), f"input recipe drifted for {case}"
    return x


def same_bits(a: np.ndarray, b: np.ndarray) -> bool:
    """Bit-identical, except that any NaN equals any NaN."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    an, bn = np.isnan(a), np.isnan(b)
    if not np.array_equal(an, bn):
        return False
    return bool(np.array_equal(a.view(np.uint32)[~an], b.view(np.uint32)[~bn]))


def check_output(case: str, rec: Dict[str, np.ndarray], out: np.ndarray) -> bool:
    if "out" in rec:
        return same_bits(out, rec["out"])
    return sha(out) == str(rec["sha_out"])


def seed_all(seed: int) -> None:
    """fl_sim/utils/misc.py:210-211 (the two streams the codec consumes)."""
    random.seed(seed)
    np.random.seed(seed)


def dense_params(name: str):
    """(kind, levels, p, fp64_stats) of a dense dithering case name."""
    if name.startswith("std_L"):
        L, pn = name[5:].split("_")
        return "std", int(L), (np.inf if pn == "inf" else 2), False
    table = {
        "natdither32_s8_inf": ("nat", 8, np.inf, False),
        "natdither64_s3_p2": ("nat", 3, 2, True),
        "stddither32_s8_inf": ("std", 8, np.inf, False),
        "stddither64_s4_inf": ("std", 4, np.inf, True),
    }
    return table[name]


def oracle_dense(name: str, x: np.ndarray) -> Tuple[np.ndarray, float]:
    """Run the oracle for a dense case with the global streams (caller seeds them)."""
    stream = ref.python_random_stream()
    if name == "identical":
        out, send = ref.identical(x)
        return out, send
    if name.startswith("lazy"):
        P = 0.3 if name == "lazy_p03" else 0.9
        return ref.lazy(x, P, random.random())
    if name in ("natural32", "natural64"):
        out, send, _ = ref.natural(x, stream, fp64_stats=(name == "natural64"))
        return out, send
    kind, L, p, fp64 = dense_params(name)
    if kind == "std":
        out, send, _ = ref.standard_dithering(x, L, p, stream, fp64_stats=fp64)
    else:
        out, send, _ = ref.natural_dithering(x, L, p, stream, fp64_stats=fp64)
    return out, send


def oracle_sparse(name: str, x: np.ndarray, D: int, K: int) -> Tuple[np.ndarray, float]:
    if name == "topk":
        return ref.topk(x, K)
    if name == "randk":
        S = np.arange(D)
        np.random.shuffle(S)
        return ref.randk(x, K, D, S[:K])
    if name == "adaptive":
        out, send, _ = ref.adaptive_random(x, D, np.random.random_sample())
        return out, send
    raise KeyError(name)


def order_keys(x: np.ndarray) -> np.ndarray:
    """np.argsort order as uint32 keys: -0 == +0, NaN largest (same map as the device's order_key)."""
    b = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).copy()
    b[b == 0x80000000] = 0
    k = np.where(b & np.uint32(0x80000000), ~b, b | np.uint32(0x80000000)).astype(np.uint32)
    k[np.isnan(x)] = 0xFFFFFFFF
    return k


def topk_valid(x: np.ndarray, out: np.ndarray, K: int) -> bool:
    """Tie-tolerant Top-K check (compressors.py:294-295 with an unstable argsort): elements above the
    K-th largest value are kept bit for bit, elements below are +0, and exactly K - #above of the ties
    are kept (ties equal to 0 are unobservable except through -0, so only their values are checked)."""
    if K <= 0 or K >= len(x):
        return same_bits(out, x)
    keys = order_keys(x)
    t = np.sort(keys)[len(x) - K]
    above, below, tie = keys > t, keys < t, keys == t
    xb, ob = x.view(np.uint32), out.view(np.uint32)
    if not np.array_equal(ob[above], xb[above]) and not (np.isnan(x[above]).all() and np.isnan(out[above]).all()):
        if not same_bits(out[above], x[above]):
            return False
    if np.any(ob[below] != 0):
        return False
    kept = (ob[tie] == xb[tie]) | (np.isnan(out[tie]) & np.isnan(x[tie]))
    zeroed = ob[tie] == 0
    if not np.all(kept | zeroed):
        return False
    if x[tie][0] == 0:
        return True
    return int(kept.sum()) == K - int(above.sum())
