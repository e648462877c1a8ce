"""The drop-in ``Compressor``'s non-codec surface against the reference itself (CPU, no GPU).

tests/golden/dropin_surface.json was written by running the reference's own factories
(``tests/golden/gen_golden.py extra``; compressors.py:58-262): ``name``/``fullName`` (including the
``"?"`` a STANDARD_DITHERING_FP32 compressor returns), ``w``/``getW()``, ``is_biased``, the compressor
name and type, the level tables, ``str``/``repr``, and what an unconstructible standard-dithering level
count (> 10) does: AssertionError after the type and table were already switched.
"""

import json
import os

import numpy as np
import pytest

from fl_sim_amd import Compressor, CompressorType

SURFACE = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dropin_surface.json")))


def _norm():
    nc = Compressor("norm")
    nc.makeIdenticalCompressor()
    return nc


def _factory(key: str):
    """The factory call gen_golden.gen_surface made for ``key``."""
    parts = key.split("_")
    head = parts[0]
    if key == "fresh":
        return lambda c: None
    if head == "identical":
        return lambda c: c.makeIdenticalCompressor()
    if head == "lazy":
        return lambda c: c.makeLazyCompressor(float(parts[1]))
    if head == "randk":
        return lambda c: c.makeRandKCompressor(int(parts[1]), int(parts[2]))
    if head == "topk":
        return lambda c: c.makeTopKCompressor(int(parts[1]), int(parts[2]))
    if head in ("natural64", "natural32"):
        return lambda c: getattr(c, f"makeNaturalCompressorFP{head[-2:]}")()
    if head == "adaptive":
        return lambda c: c.makeAdaptiveRandomCompressor(int(parts[1]))
    if head == "qsgd64":
        return lambda c: c.makeQSGD_FP64(int(parts[1]), int(parts[2]))
    if head.startswith("std"):
        fp, L = head[3:], int(parts[1])
        p = np.inf if parts[2] in ("inf", "assert") else 2
        return lambda c: getattr(c, f"makeStandardDitheringFP{fp}")(L, _norm(), p)
    if head.startswith("natd"):
        fp, L, dim = head[4:], int(parts[1]), int(parts[2])
        p = np.inf if parts[3] == "inf" else float(parts[3])
        return lambda c: getattr(c, f"makeNaturalDitheringFP{fp}")(L, dim, p)
    raise KeyError(key)


def _snap(c):
    d = {"type": c.compressorType.value, "compressorName": c.compressorName, "w": float(c.w),
         "getW": float(c.getW()), "is_biased": bool(c.is_biased), "is_unbiased": bool(c.is_unbiased),
         "name": c.name, "fullName": c.fullName, "str": str(c), "repr": repr(c)}
    if hasattr(c, "levelsValues"):
        d["levelsValues"] = [float(v) for v in np.asarray(c.levelsValues)]
        d["s"] = int(c.s)
    return d


@pytest.mark.parametrize("key", sorted(SURFACE))
def test_surface_matches_reference(key):
    want = dict(SURFACE[key])
    err = want.pop("error", None)
    c = Compressor("start")
    if key.endswith("_assert"):
        c.makeTopKCompressor(5, 50)
        with pytest.raises(AssertionError):
            _factory(key)(c)
        assert err == "AssertionError"
    else:
        _factory(key)(c)
    got = _snap(c)
    assert got == want


def test_every_type_is_covered():
    seen = {v["type"] for v in SURFACE.values()}
    assert seen == {t.value for t in CompressorType}


@pytest.mark.parametrize("levels", [11, 16, 127])
def test_extended_levels_is_opt_in(levels):
    c = Compressor(extended_levels=True)
    c.makeStandardDitheringFP32(levels, _norm())
    assert c.s == levels and c.levelsValues[-1] == 1.0 and len(c.levelsValues) == levels + 1
    assert np.array_equal(c.levelsValues, np.arange(levels + 1) * (1.0 / levels) * (np.arange(levels + 1) < levels)
                          + (np.arange(levels + 1) == levels))
    with pytest.raises(AssertionError):
        Compressor().makeStandardDitheringFP32(levels, _norm())
