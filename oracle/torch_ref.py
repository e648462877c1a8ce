"""ORACLE — test infrastructure only.  Never imported by the product package (fl_sim_amd/).

The CPU-PyTorch path of the stacked codec (BASELINE.json north_star: "the CPU-PyTorch path is timed on the
GPU box's own host cores"), used by ``bench.py``'s ``cpu_baseline`` leg: what an fl-sim user gets by running
the reference's two compressors back to back with torch tensors on the host —

* Top-K (compressors.py:293-296): ``torch.topk`` of the k largest signed values, indices sorted ascending;
* standard dithering, s levels, p = inf (compressors.py:327-365) of the kept values: y = |v| / max|v|,
  bracket s = floor(y * s), p_down = (y - lv[s+1]) / (lv[s] - lv[s+1]) in fp64, one uniform per kept value,
  the 8-bit code sign << 7 | level;
* decode: a dense zero vector with ``out[idx] = fp32(fp32(level / s) * sign) * norm``.

The uniforms come from a torch CPU generator (not the device's Philox stream) and torch.topk breaks ties
its own way, so this path is a timing baseline, not a parity oracle (``compressors_ref.stacked`` is that).
"""

from __future__ import annotations

import torch


def stacked_encode(x: torch.Tensor, k: int, levels: int, gen: torch.Generator):
    vals, idx = torch.topk(x, k, sorted=False)
    idx, order = torch.sort(idx)
    vals = vals[order]
    norm = vals.abs().max()
    y = (vals.abs() / norm).double()
    lo = torch.clamp(torch.floor(y * levels), max=levels - 1)
    lv_lo = lo / levels
    lv_hi = (lo + 1) / levels
    p_down = (y - lv_hi) / (lv_lo - lv_hi)
    u = torch.rand(k, generator=gen, dtype=torch.float64)
    level = torch.where(u < p_down, lo, lo + 1).to(torch.uint8)
    codes = level | (torch.signbit(vals).to(torch.uint8) << 7)
    return idx.to(torch.int32), codes, norm


def stacked_decode(idx: torch.Tensor, codes: torch.Tensor, norm: torch.Tensor, n: int, levels: int) -> torch.Tensor:
    level = (codes & 0x7F).to(torch.float32)
    sign = torch.where((codes >> 7).bool(), -1.0, 1.0)
    out = torch.zeros(n, dtype=torch.float32)
    out[idx.long()] = ((level.double() * (1.0 / levels)).float() * sign) * norm
    return out


def stacked_step(x: torch.Tensor, k: int, levels: int, gen: torch.Generator) -> torch.Tensor:
    idx, codes, norm = stacked_encode(x, k, levels, gen)
    return stacked_decode(idx, codes, norm, x.numel(), levels)


def dither_step(X: torch.Tensor, levels: int, gen: torch.Generator) -> torch.Tensor:
    """configs[1]'s codec on the host: standard dithering, s levels, p = inf (compressors.py:327-365) of each row of
    a [clients, d] batch — y = |x| / max|x| per row, the fp64 bracket and p_down, one uniform per element, the code
    as sign << 7 | level — and its decode ``fp32(fp32(level / s) * sign) * norm`` (zeros stay zero)."""
    norm = X.abs().amax(dim=1, keepdim=True)
    y = (X.abs() / norm).double()
    lo = torch.clamp(torch.floor(y * levels), max=levels - 1)
    p_down = (y - (lo + 1) / levels) / (lo / levels - (lo + 1) / levels)
    u = torch.rand(X.shape, generator=gen, dtype=torch.float64)
    level = torch.where(u < p_down, lo, lo + 1)
    codes = level.to(torch.uint8) | (torch.signbit(X).to(torch.uint8) << 7)
    lv = ((codes & 0x7F).double() * (1.0 / levels)).float()
    return torch.where(X == 0, torch.zeros_like(X), torch.where((codes >> 7).bool(), -lv, lv) * norm)


def topk_step(x: torch.Tensor, k: int) -> torch.Tensor:
    """configs[2]'s codec on the host: Top-K (compressors.py:293-296) by ``torch.topk`` and the dense decode."""
    vals, idx = torch.topk(x, k, sorted=False)
    out = torch.zeros_like(x)
    out[idx] = vals
    return out


def round_fold(xs, weights, k: int, levels: int, gen: torch.Generator) -> torch.Tensor:
    """configs[3]'s round on the host: every client's stacked encode + decode, folded in client order with the
    reference's ``add_(alpha=w)`` (nodes.py:1176-1180)."""
    out = torch.zeros_like(xs[0])
    for x, w in zip(xs, weights):
        out.add_(stacked_step(x, k, levels, gen), alpha=w)
    return out
