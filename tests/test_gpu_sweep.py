"""Seeded randomized sweep of the codec kernels against the oracle (gfx950): sizes drawn log-uniformly from 1 to a few
million (block-step boundaries and odd tails included), k from one element to all but one, and input families that
stress the select and the dithering — gaussian, heavy-tailed, quantized (mass ties), per-layer scales (a real model
delta), sparse (most elements exactly zero), and ±0 / ±inf / NaN sprinkled in.  Every case is bit-exact:

* top-k: the kept index set and values (stable tie rule, App. A.1);
* stacked top-k -> dithering: indices, codes, norm, tile pointers and the decoded vector;
* standard / natural dithering in Philox mode (p = inf and 2, the device norm): decoded rows and nonzero counts;
* the natural compressor;
* a round's clients: the batched stacked encode against one encode per client, the delta-fused encode over random
  tensor lists against flatten + encode, and the one-pass wire fold with random weights and client orders against
  the per-client weighted decode-accumulate chain.

The case list is fixed by its seed, so a failure names a reproducible (family, n, k, seed)."""

import math

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc

pytestmark = pytest.mark.gpu
DEV = "cuda"
FAMILIES = ("gauss", "cauchy", "ties", "layers", "sparse", "specials")


def _codec():
    from fl_sim_amd import codec

    return codec


def make_input(family: str, n: int, g: np.random.Generator, finite: bool = False) -> np.ndarray:
    if family == "gauss":
        x = g.standard_normal(n) * 1e-3
    elif family == "cauchy":
        x = g.standard_cauchy(n) * 1e-4
    elif family == "ties":  # a handful of distinct values: the k-th value is shared by many elements
        x = g.integers(-6, 7, n) * 0.25e-3
    elif family == "layers":  # tensors of very different scales laid end to end
        x = g.standard_normal(n)
        cuts = np.sort(g.integers(0, n + 1, 7))
        for a, b in zip(np.r_[0, cuts], np.r_[cuts, n]):
            x[a:b] *= 10.0 ** g.uniform(-6, 0)
    elif family == "sparse":  # most elements exactly zero (±0)
        x = g.standard_normal(n) * 1e-2
        x[g.random(n) < 0.9] = 0.0
        x[g.random(n) < 0.3] *= -0.0
    else:  # specials
        x = g.standard_normal(n) * 1e-3
        x[g.random(n) < 0.02] = 0.0
        x[g.random(n) < 0.01] = -0.0
        if not finite:
            x[g.random(n) < 0.001] = np.inf
            x[g.random(n) < 0.001] = -np.inf
            x[g.random(n) < 0.001] = np.nan
    return np.ascontiguousarray(x.astype(np.float32))


def _sizes(seed: int, count: int, hi: float):
    g = np.random.default_rng(seed)
    out = []
    for i in range(count):
        n = int(round(math.exp(g.uniform(0.0, math.log(hi)))))
        if i % 5 == 1:  # around a multiple of the encoder's 16 K-element block step
            n = int(g.integers(1, 200)) * 16384 + int(g.integers(-3, 4))
        out.append(max(n, 2))
    return out


def _k_for(n: int, g: np.random.Generator) -> int:
    """0 < k < n, the codec's range (k = 0 and k = n, the reference's keep-everything cases, are the Compressor's)"""
    r = g.random()
    if r < 0.1:
        return 1
    if r < 0.15:
        return n - 1
    return int(min(n - 1, max(1, round(n * 10.0 ** g.uniform(-4, -0.3)))))


TOPK_CASES = [(FAMILIES[i % len(FAMILIES)], n, 1000 + i) for i, n in enumerate(_sizes(11, 48, 4e6))]


@pytest.mark.parametrize("family,n,seed", TOPK_CASES)
def test_topk_sweep_vs_oracle(family, n, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, n, g)
    k = _k_for(n, g)
    idx, val, tiles = codec.topk_encode(torch.from_numpy(x).to(DEV), k, with_tiles=True)
    exp_idx, exp_val = ref.topk_kept(x, k)
    assert np.array_equal(idx.cpu().numpy().astype(np.int64), exp_idx), (family, n, k, seed)
    assert gc.same_bits(val.cpu().numpy(), exp_val)
    t = tiles.cpu().numpy().astype(np.int64)
    assert t[-1] == k and np.array_equal(t[:-1], np.searchsorted(exp_idx, np.arange(len(t) - 1) * codec.TILE))
    dense = codec.sparse_decode(idx, val, n, tiles=tiles).cpu().numpy()
    exp_dense, _ = ref.topk(x, k)
    assert gc.same_bits(dense, exp_dense)


STACKED_CASES = [(FAMILIES[(i + 2) % len(FAMILIES)], n, 2000 + i, (127, 7, 3, 1)[i % 4])
                 for i, n in enumerate(_sizes(12, 40, 4e6))]


@pytest.mark.parametrize("family,n,seed,levels", STACKED_CASES)
def test_stacked_sweep_vs_oracle(family, n, seed, levels):
    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, n, g, finite=True)  # (a NaN / inf in the kept set makes the norm non-finite)
    k = _k_for(n, g)
    pkt = codec.stacked_encode(torch.from_numpy(x).to(DEV), k, levels, seed=seed, counter=3)
    u_all = ref.philox_uniforms(n, seed, 3)
    exp_out, exp_idx, exp_codes, pn = ref.stacked(x, k, levels, lambda idx: u_all[idx])
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx), (family, n, k, seed)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), exp_codes)
    assert gc.same_bits(pkt.norm.cpu().numpy(), np.array([pn], dtype=np.float32))
    t = pkt.tiles.cpu().numpy().astype(np.int64)
    assert t[-1] == k and np.array_equal(t[:-1], np.searchsorted(exp_idx, np.arange(len(t) - 1) * codec.TILE))
    assert gc.same_bits(codec.stacked_decode(pkt).cpu().numpy(), exp_out)


def _quant_cases():
    g = np.random.default_rng(13)
    cases = []
    for i in range(36):
        rows = int(g.integers(1, 12))
        d = int(round(math.exp(g.uniform(0.0, math.log(600_000)))))
        kind, levels = (("std", 127), ("std", 5), ("nat", 8), ("std", 1), ("nat", 2), ("std", 10))[i % 6]
        p = math.inf if i % 3 else 2.0
        cases.append((FAMILIES[i % len(FAMILIES)], rows, max(d, 1), kind, levels, p, 3000 + i))
    return cases


@pytest.mark.parametrize("family,rows,d,kind,levels,p,seed", _quant_cases())
def test_quant_sweep_vs_oracle(family, rows, d, kind, levels, p, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, rows * d, g, finite=True).reshape(rows, d)
    xd = torch.from_numpy(x).to(DEV)
    norms = codec.quant_norm(xd, p)
    pkt = codec.quant_encode(xd, 0 if kind == "std" else 1, levels, norms, seed, 5, None, want_nnz=True)
    out = codec.quant_decode(pkt).cpu().numpy()
    lv = ref.standard_levels(levels) if kind == "std" else ref.natural_levels(levels)
    u_all = ref.philox_uniforms(rows * d, seed, 5)
    nr = norms.cpu().numpy()
    if math.isinf(p):
        assert np.array_equal(nr, np.abs(x).max(axis=1))
    for r in range(rows):
        u_row = u_all[r * d:(r + 1) * d]
        exp, nnz, _, _ = ref.dither(x[r], lv, nr[r], lambda idx: u_row[idx])
        assert gc.same_bits(out[r], exp), (family, rows, d, kind, levels, p, seed, r)
        assert int(pkt.nnz[r].item()) == nnz
    # the one-call form (norms computed inside, decode fused) equals the separate calls
    if math.isinf(p):
        pk2, out2 = codec.quant_encode_auto(xd, 0 if kind == "std" else 1, levels, seed=seed, counter=5)
        assert torch.equal(pk2.norms, norms)
        assert gc.same_bits(out2.cpu().numpy(), out)


@pytest.mark.parametrize("family,n,seed", [(FAMILIES[i % len(FAMILIES)], n, 4000 + i)
                                           for i, n in enumerate(_sizes(14, 24, 2e6))])
def test_natural_sweep_vs_oracle(family, n, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    x = make_input(family, n, g, finite=True)
    codes, nnz = codec.natural_encode(torch.from_numpy(x).to(DEV), seed, 2)
    out = codec.natural_decode(codes, n).cpu().numpy()
    u_all = ref.philox_uniforms(n, seed, 2)
    exp, _, nz = ref.natural(x, lambda idx: u_all[idx])
    assert gc.same_bits(out, exp), (family, n, seed)
    assert int(nnz.item()) == nz


def _same_packet(a, b):
    k = a.idx.numel()
    return (torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k])
            and torch.equal(a.norm.view(torch.int32), b.norm.view(torch.int32))
            and (a.tiles is None or b.tiles is None or torch.equal(a.tiles, b.tiles)))


def _batch_cases():
    g = np.random.default_rng(15)
    out = []
    for i in range(10):
        C = int(g.integers(1, 40))
        n = int(round(math.exp(g.uniform(math.log(2000), math.log(3e6 / C)))))
        out.append((C, n, 5000 + i))
    return out


@pytest.mark.parametrize("C,n,seed", _batch_cases())
def test_batch_sweep_equals_single_encodes(C, n, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    k = _k_for(n, g)
    xs = [torch.from_numpy(make_input(FAMILIES[(c + seed) % len(FAMILIES)], n, g, finite=True)).to(DEV)
          for c in range(C)]
    seeds = [int(v) for v in g.integers(0, 1 << 30, C)]
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=seeds, counter=seed)
    for c in range(C):
        assert _same_packet(pks[c], codec.stacked_encode(xs[c], k, 127, seed=seeds[c], counter=seed)), (C, n, k, c)


def _delta_cases():
    g = np.random.default_rng(16)
    out = []
    for i in range(10):
        T = int(g.integers(1, 80))
        sizes = [int(round(math.exp(g.uniform(0, math.log(200_000))))) for _ in range(T)]
        sizes[int(g.integers(0, T))] = 0 if T > 1 else sizes[0]  # an empty tensor somewhere
        out.append((sizes, 6000 + i))
    return out


@pytest.mark.parametrize("sizes,seed", _delta_cases())
def test_delta_sweep_equals_flatten_then_encode(sizes, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    n = sum(sizes)
    if n < 2:
        pytest.skip("a single element has no 0 < k < n")
    glo = [torch.from_numpy(make_input("gauss", s, g) * 100).to(DEV) for s in sizes]
    loc = [gl + torch.from_numpy(make_input(FAMILIES[i % len(FAMILIES)], s, g, finite=True)).to(DEV)
           for i, (gl, s) in enumerate(zip(glo, sizes))]
    k = _k_for(n, g)
    a = codec.stacked_encode_delta(loc, glo, k, 127, seed=seed, counter=1)
    b = codec.stacked_encode(codec.delta_flatten(loc, glo), k, 127, seed=seed, counter=1)
    assert _same_packet(a, b), (len(sizes), n, k)


@pytest.mark.parametrize("m,n,seed", [(int(m), int(n), 7000 + i) for i, (m, n) in enumerate(
    zip(np.random.default_rng(17).integers(1, 40, 8), np.random.default_rng(18).integers(1000, 400_000, 8)))])
def test_wire_fold_sweep_equals_decode_accumulate_chain(m, n, seed):
    codec = _codec()
    g = np.random.default_rng(seed)
    k = _k_for(n, g)
    stride, _ = codec.stacked_wire_layout(n, k)
    recs = torch.zeros(m, stride, dtype=torch.uint8, device=DEV)
    for i in range(m):
        x = torch.from_numpy(make_input(FAMILIES[i % len(FAMILIES)], n, g, finite=True)).to(DEV)
        codec.stacked_encode(x, k, 127, seed=seed + i, counter=2, wire=recs[i])
    slots = [int(v) for v in g.permutation(m)]
    weights = [float(v) for v in (g.random(m) - 0.3) * 0.5]  # signs mixed
    exp = torch.zeros(n, device=DEV)
    for s, w in zip(slots, weights):
        codec.stacked_decode(codec.wire_packet(recs[s], n, k), out=exp, weight=w, accumulate=True)
    got = codec.stacked_fold_wires(recs, slots, weights, n, k)
    assert torch.equal(got.view(torch.int32), exp.view(torch.int32)), (m, n, k)
