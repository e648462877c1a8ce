"""Seeded randomized sweep of the float64 codec (f64.hip, adaptive.hip on float64) against the oracle (gfx950).

Sizes drawn log-uniformly from 1 to a few million with the 8192-element chunk boundaries and odd tails included; input
families that stress each kernel in float64 — gaussian, heavy-tailed, quantized (mass ties), per-layer scales spanning
the float64 exponent range (1e-300 … 1e300), sparse (most elements ±0), subnormals, and the specials.  Every case is
bit-exact against the oracle fed the same Philox uniforms:

* top-k: the dense output (stable tie rule: the highest indices among ties), k from 1 to n - 1;
* natural compression: codes' decoded vector;
* standard / natural dithering at p = inf and 2 (the device norm, passed to the oracle), the decoded vector and the
  nonzero count;
* adaptive random: the index and the dense output for three uniforms.

The case list is fixed by its seed, so a failure names a reproducible (family, n, seed)."""

import math

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_f64 as g64

pytestmark = pytest.mark.gpu
DEV = "cuda"
FAMILIES = ("gauss", "cauchy", "ties", "layers", "sparse", "subnormal", "specials")


def _codec():
    from fl_sim_amd import codec

    return codec


def make_input(family: str, n: int, g: np.random.Generator, finite: bool = True) -> np.ndarray:
    if family == "gauss":
        x = g.standard_normal(n) * 1e-3
    elif family == "cauchy":
        x = g.standard_cauchy(n) * 1e-4
    elif family == "ties":
        x = g.integers(-6, 7, n) * 0.25e-3
    elif family == "layers":  # tensors of very different scales, across the float64 exponent range
        x = g.standard_normal(n)
        cuts = np.sort(g.integers(0, n + 1, 7))
        for a, b in zip(np.r_[0, cuts], np.r_[cuts, n]):
            x[a:b] *= 10.0 ** g.uniform(-300, 300)
    elif family == "sparse":
        x = g.standard_normal(n) * 1e-2
        x[g.random(n) < 0.9] = 0.0
        x[g.random(n) < 0.3] *= -0.0
    elif family == "subnormal":  # float64 subnormals and their neighbours
        x = g.standard_normal(n) * 1e-310
        x[g.random(n) < 0.2] *= 1e10
    else:
        x = g.standard_normal(n) * 1e-3
        x[g.random(n) < 0.02] = 0.0
        x[g.random(n) < 0.01] = -0.0
        if not finite:
            x[g.random(n) < 0.001] = np.inf
            x[g.random(n) < 0.001] = -np.inf
            x[g.random(n) < 0.001] = np.nan
    return np.ascontiguousarray(x.astype(np.float64))


def _sizes(seed: int, count: int, hi: float):
    g = np.random.default_rng(seed)
    out = []
    for i in range(count):
        n = int(round(math.exp(g.uniform(0.0, math.log(hi)))))
        if i % 4 == 1:  # around a multiple of the 8192-element chunk
            n = int(g.integers(1, 300)) * 8192 + int(g.integers(-3, 4))
        out.append(max(n, 2))
    return out


def _k_for(n: int, g: np.random.Generator) -> int:
    r = g.random()
    if r < 0.1:
        return 1
    if r < 0.15:
        return n - 1
    return int(min(n - 1, max(1, round(n * 10.0 ** g.uniform(-4, -0.3)))))


TOPK_CASES = [(FAMILIES[i % len(FAMILIES)], n, 5000 + i) for i, n in enumerate(_sizes(21, 42, 3e6))]


@pytest.mark.parametrize("family,n,seed", TOPK_CASES)
def test_topk_f64_sweep_vs_oracle(family, n, seed):
    g = np.random.default_rng(seed)
    x = make_input(family, n, g, finite=False)
    k = _k_for(n, g)
    got = _codec().topk_dense_f64(torch.from_numpy(x).to(DEV), k).cpu().numpy()
    exp, _ = ref.topk(x, k)
    assert g64.same_bits(got, exp), (family, n, k, seed)


NAT_CASES = [(FAMILIES[(i + 1) % len(FAMILIES)], n, 6000 + i) for i, n in enumerate(_sizes(22, 21, 3e6))]


@pytest.mark.parametrize("family,n,seed", NAT_CASES)
def test_natural_f64_sweep_vs_oracle(family, n, seed):
    g = np.random.default_rng(seed)
    x = make_input(family, n, g)
    codes, out = _codec().natural_f64(torch.from_numpy(x).to(DEV), seed=seed, counter=4, want_codes=True)
    exp, _, _ = ref.natural64(x, ref.philox_stream(seed, 4, n))
    assert g64.same_bits(out.cpu().numpy(), exp), (family, n, seed)
    assert g64.same_bits(_codec().natural_decode_f64(codes, n).cpu().numpy(), exp)


def _quant_cases():
    g = np.random.default_rng(23)
    out = []
    for i, n in enumerate(_sizes(24, 30, 2e6)):
        kind, levels = (("std", 127), ("std", 5), ("nat", 8), ("std", 1), ("nat", 2), ("std", 10))[i % 6]
        out.append((FAMILIES[i % len(FAMILIES)], n, kind, levels, math.inf if i % 3 else 2.0, 7000 + i))
    return out


@pytest.mark.parametrize("family,n,kind,levels,p,seed", _quant_cases())
def test_dithering_f64_sweep_vs_oracle(family, n, kind, levels, p, seed):
    from fl_sim_amd._lib import FLC_Q_NATURAL_DITHER, FLC_Q_STANDARD_DITHER

    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, n, g)
    xd = torch.from_numpy(x).to(DEV)
    norm = codec.quant_norm_f64(xd, p)
    pn = np.float64(norm.item())
    kd = FLC_Q_STANDARD_DITHER if kind == "std" else FLC_Q_NATURAL_DITHER
    levels_tab = ref.standard_levels(levels) if kind == "std" else ref.natural_levels(levels)
    try:
        exp, nz, _, _ = ref.dither64(x, levels_tab, pn, ref.philox_stream(seed, 5, n))
    except IndexError:  # a p = 2 norm underflowed to 0 under nonzero elements (the reference raises; not a codec case)
        assert pn == 0.0
        return
    _, out, nnz = codec.quant_f64(xd, kd, levels, norm, seed=seed, counter=5, want_nnz=True)
    assert g64.same_bits(out.cpu().numpy(), exp), (family, n, kind, levels, p, seed)
    assert int(nnz.item()) == nz


ADAPTIVE_CASES = [(FAMILIES[(i + 3) % len(FAMILIES)], n, 8000 + i) for i, n in enumerate(_sizes(25, 14, 3e6))]


@pytest.mark.parametrize("family,n,seed", ADAPTIVE_CASES)
def test_adaptive_f64_sweep_vs_oracle(family, n, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, n, g)
    if family == "sparse":
        x[0] = 1e-3  # at least one nonzero
    xd = torch.from_numpy(x).to(DEV)
    status = int(codec.adaptive_prepare(xd).item())
    with np.errstate(all="ignore"):
        p = np.abs(x) / np.abs(x).sum()
    exp_status = 1 if np.isnan(p.sum()) else (2 if abs(p.sum() - 1.0) > np.sqrt(np.finfo(np.float64).eps) else 0)
    assert status == exp_status, (family, n, seed)
    if status:
        return
    for u in (0.0, float(g.random()), 1.0 - 2.0**-53):
        out, index = codec.adaptive_select(xd, u)
        exp, _, ind = ref.adaptive_random(x, n, u)
        assert int(index.item()) == ind, (family, n, seed, u)
        assert g64.same_bits(out.cpu().numpy(), exp)
