"""GPU parity of the codec kernels (gfx950) against the reference fixtures and the oracle.

* compat RNG: the drop-in ``Compressor`` on numpy inputs reproduces the reference's own outputs
  (tests/golden) bit for bit, its send statistics, and leaves the global random streams where the
  reference leaves them;
* philox RNG: the kernels match the oracle fed the same Philox uniforms, bit for bit;
* top-k: exact kept sets (stable tie rule) at sizes up to 25M, fallback path, ties, NaN/+-0, skew;
* full size (BASELINE configs): size-independent properties of the stacked codec on 1 GiB.
"""

import math
import random

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc

pytestmark = pytest.mark.gpu

DENSE = gc.load("codec_dense.npz")
SPARSE = gc.load("codec_sparse.npz")
DEV = "cuda"


def _codec():
    from fl_sim_amd import codec

    return codec


def make_compressor(name, rng="compat", seed=0):
    from fl_sim_amd import Compressor

    c = Compressor(rng=rng, seed=seed)
    if name == "identical":
        c.makeIdenticalCompressor()
    elif name.startswith("lazy"):
        c.makeLazyCompressor(0.3 if name == "lazy_p03" else 0.9)
    elif name == "natural32":
        c.makeNaturalCompressorFP32()
    elif name == "natural64":
        c.makeNaturalCompressorFP64()
    else:
        kind, L, p, fp64 = gc.dense_params(name)
        if kind == "std":
            nc = Compressor("norm")
            nc.makeIdenticalCompressor()
            (c.makeStandardDitheringFP64 if fp64 else c.makeStandardDitheringFP32)(L, nc, p)
        else:
            (c.makeNaturalDitheringFP64 if fp64 else c.makeNaturalDitheringFP32)(L, 100, p)
    return c


def _is_p2(name):
    return name.endswith("_p2")


@pytest.mark.parametrize("case", sorted(DENSE))
def test_dense_compressor_matches_reference_fixture(case):
    rec = DENSE[case]
    name, _, seed = case.split("|")
    x = gc.case_input(case, rec)
    c = make_compressor(name)
    gc.seed_all(int(seed))
    out = c.compressVector(x)
    assert isinstance(out, np.ndarray) and out.dtype == np.float32 and out.shape == x.shape
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])
    assert float(c.last_need_to_send_advance) == float(rec["send"])
    assert c.total_input_components == len(x)
    # p = 2 included: compat mode on a host input takes the reference's own np.linalg.norm (norm="auto")
    assert gc.check_output(case, rec, out), case
    if _is_p2(name) and "out" in rec:
        # the device norm (norm="device": an fp64 sum of squares rounded once) stays within north_star's 1e-6
        cd = make_compressor(name)
        cd.norm_mode = "device"
        gc.seed_all(int(seed))
        np.testing.assert_allclose(cd.compressVector(x), rec["out"], rtol=1e-6, atol=0)


@pytest.mark.parametrize("case", [k for k in sorted(DENSE) if _is_p2(k.split("|")[0]) and "x" in DENSE[k]])
def test_dense_l2_with_reference_norm_is_bit_exact(case):
    codec = _codec()
    rec = DENSE[case]
    name, _, seed = case.split("|")
    kind, L, p, fp64 = gc.dense_params(name)
    x = gc.case_input(case, rec)
    gc.seed_all(int(seed))
    pn = ref.vector_norm(x, 2)  # what the reference computes (np.linalg.norm)
    xd = torch.from_numpy(x).to(DEV).reshape(1, -1)
    norms = torch.tensor([pn], dtype=torch.float32, device=DEV)
    cnt = int(codec.count_consumers(xd, norms).item())
    from fl_sim_amd import rng

    u = torch.from_numpy(rng.python_random_doubles(cnt)).to(DEV)
    pkt = codec.quant_encode(xd, 0 if kind == "std" else 1, L, norms, compat_u=u)
    out = codec.quant_decode(pkt).reshape(-1).cpu().numpy()
    assert gc.same_bits(out, rec["out"])
    # and our own device L2 norm is within 2 ulp of the exact one
    exact = np.float32(np.sqrt(np.sum(x.astype(np.float64) ** 2)))
    ours = codec.quant_norm(xd, 2).item()
    assert abs(ours - exact) <= 2 * np.spacing(exact)


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("D", [4_000_000, 25_000_000])
@pytest.mark.parametrize("kind", ["std", "nat"])
def test_dense_l2_compat_large_d_matches_oracle(D, kind, where):
    """p = 2 at realistic D through the drop-in Compressor (compat mode, numpy input): the norm is the reference's
    own np.linalg.norm (an fp32 BLAS dot, 3e-6 .. 6e-5 away from the exact norm at these sizes), so the output
    equals the oracle's, which calls np.linalg.norm on this same host, bit for bit.  ``device``: the same vector as a
    HIP tensor, where the default norm="auto" also takes the reference's norm (round 4)."""
    from fl_sim_amd import Compressor

    g = np.random.default_rng(D + (kind == "nat"))
    x = (g.standard_normal(D) * 1e-3).astype(np.float32)
    x[g.random(D) < 0.05] = 0
    c = Compressor()
    if kind == "std":
        nc = Compressor("norm")
        nc.makeIdenticalCompressor()
        c.makeStandardDitheringFP32(8, nc, 2)
    else:
        c.makeNaturalDitheringFP32(8, D, 2)
    random.seed(17)
    got = c.compressVector(x if where == "host" else torch.from_numpy(x).to(DEV))
    if where == "device":
        assert got.device.type == "cuda"
        got = got.cpu().numpy()
    after = random.random()
    random.seed(17)
    fn = ref.standard_dithering if kind == "std" else ref.natural_dithering
    want, send, pn = fn(x, 8, 2, ref.python_random_stream())
    assert random.random() == after  # the same number of uniforms consumed
    assert gc.same_bits(got, want)
    assert float(c.last_need_to_send_advance) == float(send)
    # the device norm (norm="device") is the exact norm to 1 ulp; the reference's differs from it at this size
    exact = np.float32(np.sqrt(np.sum(x.astype(np.float64) ** 2)))
    dn = _codec().quant_norm(torch.from_numpy(x).to(DEV).reshape(1, -1), 2).item()
    assert abs(dn - exact) <= 2 * np.spacing(exact)
    assert pn == np.float32(np.linalg.norm(x, 2))


@pytest.mark.parametrize("case", sorted(SPARSE))
def test_sparse_compressor_matches_reference_fixture(case):
    from fl_sim_amd import Compressor

    rec = SPARSE[case]
    parts = case.split("|")
    name, seed = parts[0], int(parts[-1])
    x = gc.case_input(case, rec)
    D = len(x)
    K = 1 if name == "adaptive" else int(parts[2])
    c = Compressor()
    if name == "adaptive":
        c.makeAdaptiveRandomCompressor(D)
    elif name == "topk":
        c.makeTopKCompressor(K, D)
    else:
        K = max(K, 1)
        c.makeRandKCompressor(K, D)
    gc.seed_all(seed)
    out = c.compressVector(x)
    if name == "topk":
        assert gc.topk_valid(x, out, K), case
        expect, _ = ref.topk(x, K)  # stable rule: exact
        assert gc.same_bits(out, expect)
    else:
        assert gc.check_output(case, rec, out), case
    assert float(c.last_need_to_send_advance) == float(rec["send"])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


@pytest.mark.parametrize("kind,levels", [(0, 127), (0, 7), (1, 8), (0, 1), (1, 3)])
@pytest.mark.parametrize("rows,d,compat", [(10, 417482, False), (3, 1001, True), (1, 13, True), (2, 8192 * 3 + 5, False)])
def test_quant_encode_decode_equals_encode_then_decode(kind, levels, rows, d, compat):
    """flc_quant_encode_decode writes the codes flc_quant_encode writes and the values flc_quant_decode gives."""
    codec = _codec()
    g = np.random.default_rng(rows + d + levels)
    x = (g.standard_normal((rows, d)) * 1e-3).astype(np.float32)
    x[g.random((rows, d)) < 0.05] = 0
    xd = torch.from_numpy(x).to(DEV)
    norms = codec.quant_norm(xd)
    u = None
    if compat:
        cnt = int(codec.count_consumers(xd, norms).item())
        u = torch.from_numpy(np.random.default_rng(1).random(cnt)).to(DEV)
    pkt = codec.quant_encode(xd, kind, levels, norms, 5, 3, u, want_nnz=True)
    ref_out = codec.quant_decode(pkt)
    pkt2, out2 = codec.quant_encode_decode(xd, kind, levels, norms, 5, 3, u, want_nnz=True)
    assert torch.equal(pkt.codes, pkt2.codes) and torch.equal(pkt.nnz, pkt2.nnz)
    assert gc.same_bits(out2.cpu().numpy(), ref_out.cpu().numpy())


@pytest.mark.parametrize("p", [math.inf, 2])
@pytest.mark.parametrize("kind,levels", [(0, 127), (1, 8), (0, 3)])
@pytest.mark.parametrize("rows,d", [(10, 417482), (3, 1001), (2, 2048), (5, 4099), (1, 13), (3, 2_000_003),
                                    (1, 16384), (300, 20_000), (7, 16_387)])
def test_quant_encode_auto_equals_the_separate_calls(p, kind, levels, rows, d):
    """flc_quant_encode_auto = quant_norm + encode + decode.  p = inf at configs[1]'s shape (10 x 417,482), 3 x 2 M,
    1 x 16384 and 7 x 16387 takes the one-launch path (grid exchange of the row maxima; 2 or 4 groups per thread),
    300 x 20,000 and the rest the two-launch path (the norm partials folded inside the encode for d >= 2048)."""
    codec = _codec()
    g = np.random.default_rng(rows * 7 + d)
    x = (g.standard_normal((rows, d)) * 1e-3).astype(np.float32)
    x[g.random((rows, d)) < 0.05] = 0
    xd = torch.from_numpy(x).to(DEV)
    norms = codec.quant_norm(xd, p)
    pkt = codec.quant_encode(xd, kind, levels, norms, 9, 4, None, want_nnz=True)
    ref_out = codec.quant_decode(pkt)
    for dec in (True, False):
        pkt2, out2 = codec.quant_encode_auto(xd, kind, levels, p, 9, 4, want_nnz=True, decode=dec)
        assert gc.same_bits(pkt2.norms.cpu().numpy(), norms.cpu().numpy())
        assert torch.equal(pkt.codes, pkt2.codes) and torch.equal(pkt.nnz, pkt2.nnz)
        if dec:
            assert gc.same_bits(out2.cpu().numpy(), ref_out.cpu().numpy())
    pkt3, out3 = codec.quant_encode_auto(xd, kind, levels, p, 9, 4)  # repeated calls: no state carried over
    assert torch.equal(pkt.codes, pkt3.codes) and gc.same_bits(out3.cpu().numpy(), ref_out.cpu().numpy())


def test_raw_stream_handle_is_the_current_stream():
    """codec._stream (torch's raw current-stream accessor) names the stream torch.cuda.current_stream names: the
    default stream, a side stream under `with torch.cuda.stream`, a device given without an index."""
    codec = _codec()
    d = torch.device("cuda", 0)
    assert codec._stream(d) == torch.cuda.current_stream(d).cuda_stream
    s = torch.cuda.Stream(d)
    with torch.cuda.stream(s):
        assert codec._stream(d) == s.cuda_stream
        assert codec._stream(torch.device("cuda")) == s.cuda_stream
    assert codec._stream(torch.device("cuda")) == torch.cuda.current_stream().cuda_stream


def test_quant_one_launch_interleaved_shapes_share_the_exchange_words():
    """The one-launch quantizer's exchange words are tagged per call and polled per row: shapes with different grids
    and row layouts interleaved on one workspace (a word left by a larger grid must never pass for this call's), each
    call equal to the separate calls, and the exchange's error word 0 at the end."""
    codec = _codec()
    cases = []
    for rows, d in ((10, 417482), (1, 16384), (3, 2_000_003), (7, 16_387), (2, 1_000_000)):
        g = np.random.default_rng(rows + d)
        xd = torch.from_numpy((g.standard_normal((rows, d)) * 1e-3).astype(np.float32)).to(DEV)
        norms = codec.quant_norm(xd, math.inf)
        pkt = codec.quant_encode(xd, 0, 127, norms, 5, 1, None)
        cases.append((xd, pkt.codes.clone(), codec.quant_decode(pkt).clone()))
    codec.quant_status(reset=True)
    for rep in range(3):
        for xd, codes, out in cases[rep % 2:] + cases[: rep % 2]:
            pkt2, out2 = codec.quant_encode_auto(xd, 0, 127, math.inf, 5, 1)
            assert torch.equal(pkt2.codes, codes) and torch.equal(out2.view(torch.int32), out.view(torch.int32))
    assert codec.quant_status() == 0


def test_quant_one_launch_nan_and_zero_rows():
    """The one-launch path on rows with NaN / inf / all zeros: the norms and codes of the two-launch path."""
    codec = _codec()
    g = np.random.default_rng(3)
    x = (g.standard_normal((4, 417_482)) * 1e-3).astype(np.float32)
    x[1, 77] = np.nan
    x[2, :] = 0
    x[3, 5] = np.inf
    xd = torch.from_numpy(x).to(DEV)
    norms = codec.quant_norm(xd, math.inf)
    pkt = codec.quant_encode(xd, 0, 127, norms, 3, 1, None, want_nnz=True)
    pkt2, out2 = codec.quant_encode_auto(xd, 0, 127, math.inf, 3, 1, want_nnz=True)
    assert gc.same_bits(pkt2.norms.cpu().numpy(), norms.cpu().numpy())
    assert torch.equal(pkt.codes, pkt2.codes) and torch.equal(pkt.nnz, pkt2.nnz)
    assert gc.same_bits(out2.cpu().numpy(), codec.quant_decode(pkt).cpu().numpy())


@pytest.mark.parametrize("D,K", [(4096, 41), (1_000_003, 10_000), (25_000_000, 250_000), (100, 100), (7, 3)])
def test_randk_philox_matches_oracle(D, K):
    """Rand-K in philox mode (compressors.py:284-292): the index set is the K largest Philox keys,
    chosen on the device; equal to the oracle's restatement, and the Compressor output is D/K * x on that set."""
    from fl_sim_amd import Compressor

    codec = _codec()
    idx = codec.randk_indices(D, K, 77, 5, torch.device(DEV)).cpu().numpy().astype(np.int64)
    exp = ref.randk_philox_indices(D, K, 77, 5)
    assert np.array_equal(idx, exp)
    assert len(np.unique(idx)) == min(K, D)
    if D <= 1_000_003:
        g = np.random.default_rng(D)
        x = (g.standard_normal(D) * 1e-3).astype(np.float32)
        c = Compressor(rng="philox", seed=77)
        c.philox.counter = 5
        c.makeRandKCompressor(K, D)
        out = c.compressVector(x)
        want, send = ref.randk(x, K, D, exp)
        assert gc.same_bits(out, want) and c.last_need_to_send_advance == K


def test_randk_philox_is_uniform():
    """Each index is kept with probability K/D: 3000 draws of K = 10 from D = 100."""
    codec = _codec()
    counts = np.zeros(100)
    for c in range(3000):
        counts[codec.randk_indices(100, 10, 3, c, torch.device(DEV)).cpu().numpy()] += 1
    sigma = np.sqrt(3000 * 0.1 * 0.9)
    assert np.abs(counts - 300).max() < 5 * sigma
    assert counts.sum() == 30000


# ----------------------------------------------------------------------------------------- philox mode
@pytest.mark.parametrize("kind,levels,p", [("std", 127, math.inf), ("std", 8, math.inf), ("std", 7, 2),
                                           ("nat", 8, math.inf), ("std", 1, math.inf), ("nat", 3, 2)])
@pytest.mark.parametrize("rows,d", [(1, 4096), (10, 417482), (3, 1001), (1, 13)])
def test_quant_philox_matches_oracle(kind, levels, p, rows, d):
    codec = _codec()
    g = np.random.default_rng(rows * 1000 + d)
    x = (g.standard_normal((rows, d)) * 1e-3).astype(np.float32)
    x[g.random((rows, d)) < 0.05] = 0
    xd = torch.from_numpy(x).to(DEV)
    norms = codec.quant_norm(xd, p)
    seed, ctr = 1234, 7
    pkt = codec.quant_encode(xd, 0 if kind == "std" else 1, levels, norms, seed, ctr, None, want_nnz=True)
    out = codec.quant_decode(pkt).cpu().numpy()
    lv = ref.standard_levels(levels) if kind == "std" else ref.natural_levels(levels)
    u_all = ref.philox_uniforms(rows * d, seed, ctr)
    nr = norms.cpu().numpy()
    for r in range(rows):
        u_row = u_all[r * d:(r + 1) * d]
        exp, nnz, _, _ = ref.dither(x[r], lv, nr[r], lambda idx: u_row[idx])
        assert gc.same_bits(out[r], exp), f"row {r}"
        assert int(pkt.nnz[r].item()) == nnz
    if math.isinf(p):
        assert np.array_equal(nr, np.abs(x).max(axis=1))


def test_quant_decode_accumulate_row_weights():
    codec = _codec()
    g = np.random.default_rng(5)
    x = (g.standard_normal((4, 1000)) * 1e-2).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    pkt = codec.quant_encode(xd, 0, 127, codec.quant_norm(xd), 9, 1)
    dec = codec.quant_decode(pkt)
    w = torch.tensor([0.1, 0.2, 0.3, 0.4], device=DEV)
    acc = torch.full((4, 1000), 0.5, device=DEV)
    codec.quant_decode(pkt, out=acc, row_weights=w, accumulate=True)
    expect = np.fmaf if hasattr(np, "fmaf") else None
    d = dec.cpu().numpy().astype(np.float64)
    e = (w.cpu().numpy()[:, None].astype(np.float64) * d + 0.5).astype(np.float32)
    np.testing.assert_allclose(acc.cpu().numpy(), e, rtol=1e-7, atol=1e-9)
    scaled = codec.quant_decode(pkt, row_weights=w)
    np.testing.assert_array_equal(scaled.cpu().numpy(), (w.cpu().numpy()[:, None] * dec.cpu().numpy()))
    del expect


@pytest.mark.parametrize("n", [1, 9, 4096, 100003])
def test_natural_philox_matches_oracle(n):
    codec = _codec()
    g = np.random.default_rng(n)
    x = (g.standard_normal(n) * 10.0 ** g.integers(-30, 30, n)).astype(np.float32)
    x[g.random(n) < 0.1] = 0
    if n > 8:
        x[:6] = [1e-40, -3e-42, 1e-45, 2.0**-126, 4.0, -0.0]
    xd = torch.from_numpy(x).to(DEV)
    codes, nnz = codec.natural_encode(xd, 77, 3)
    out = codec.natural_decode(codes, n).cpu().numpy()
    u_all = ref.philox_uniforms(n, 77, 3)
    exp, _, nz = ref.natural(x, lambda idx: u_all[idx])
    assert gc.same_bits(out, exp)
    assert int(nnz.item()) == nz


# ------------------------------------------------------------------------------------------------ top-k
def _topk_device(x_np, k):
    codec = _codec()
    xd = torch.from_numpy(x_np).to(DEV)
    idx, val = codec.topk_encode(xd, k)
    return idx.cpu().numpy(), val.cpu().numpy()


def _check_topk(x, k, idx, val):
    exp_idx, exp_val = ref.topk_kept(x, k)
    assert np.array_equal(idx.astype(np.int64), exp_idx), "kept index set / order differs"
    assert gc.same_bits(val, exp_val)


@pytest.mark.parametrize("n,k", [(2, 1), (100, 1), (100, 99), (4096, 41), (65537, 655), (1 << 20, 10485),
                                 (3_000_001, 300_000), (25_000_000, 250_000)])
def test_topk_exact_random(n, k):
    g = np.random.default_rng(n + k)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    idx, val = _topk_device(x, k)
    _check_topk(x, k, idx, val)


def test_topk_ties_nan_signed_zero():
    g = np.random.default_rng(1)
    n = 300_000
    x = g.integers(-5, 6, n).astype(np.float32)  # massive ties
    x[g.random(n) < 0.01] = np.nan
    x[g.random(n) < 0.01] = -0.0
    x[g.random(n) < 0.001] = np.inf
    x[g.random(n) < 0.001] = -np.inf
    for k in (1, 2500, 3000, 50_000, 150_000, 299_999):
        idx, val = _topk_device(x, k)
        _check_topk(x, k, idx, val)


def test_topk_fallback_when_sample_misses():
    # sampled positions hold the largest values, so the candidate floor admits too few elements
    n, k, S = 4_000_000, 200_000, 32768
    x = np.full(n, 1e-6, dtype=np.float32)
    pos = ((np.arange(S) + 0.5) * n / S).astype(np.int64)
    x[pos] = 1.0
    g = np.random.default_rng(2)
    x[g.integers(0, n, 500_000)] = g.random(500_000).astype(np.float32) * 1e-3
    idx, val = _topk_device(x, k)
    _check_topk(x, k, idx, val)


def test_topk_skewed_region():
    # all of the top 1% sits in one contiguous block (per-layer scale of a real model delta)
    n = 5_000_000
    g = np.random.default_rng(3)
    x = (g.standard_normal(n) * 1e-4).astype(np.float32)
    x[1_000_000:1_100_000] *= 1000
    k = 50_000
    idx, val = _topk_device(x, k)
    _check_topk(x, k, idx, val)


def test_sparse_decode_and_accumulate():
    codec = _codec()
    g = np.random.default_rng(4)
    n, k = 1_000_003, 10_000
    x = (g.standard_normal(n)).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    idx, val = codec.topk_encode(xd, k)
    dense = codec.sparse_decode(idx, val, n).cpu().numpy()
    exp, _ = ref.topk(x, k)
    assert gc.same_bits(dense, exp)
    acc = torch.ones(n, device=DEV)
    codec.sparse_decode(idx, val, n, out=acc, weight=0.25, accumulate=True)
    e = (0.25 * exp.astype(np.float64) + 1.0).astype(np.float32)
    np.testing.assert_array_equal(acc.cpu().numpy(), e)


@pytest.mark.parametrize("n,k", [(1000, 10), (4096, 41), (1_000_003, 10_000), (25_000_000, 250_000)])
def test_topk_tiles_match_index_pass_and_decode(n, k):
    """Encoder-emitted tile pointers equal the decoder-side index pass (flc_tile_index), and the tiled
    decode equals the untiled one bit for bit (plain and accumulating)."""
    codec = _codec()
    g = np.random.default_rng(n)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    idx, val, tiles = codec.topk_encode(xd, k, with_tiles=True)
    ref_tiles = torch.empty_like(tiles)
    codec.call("flc_tile_index", codec._p(idx), k, n, codec._p(ref_tiles), codec._stream(xd.device))
    assert torch.equal(tiles, ref_tiles)
    t = tiles.cpu().numpy().astype(np.int64)
    i = idx.cpu().numpy().astype(np.int64)
    assert t[-1] == k and np.all(np.diff(t) >= 0)
    assert np.array_equal(t[:-1], np.searchsorted(i, np.arange(len(t) - 1) * codec.TILE))
    a = codec.sparse_decode(idx, val, n, tiles=tiles)
    b = codec.sparse_decode(idx, val, n)
    assert torch.equal(a, b)
    acc_a = torch.full((n,), 0.5, device=DEV)
    acc_b = acc_a.clone()
    codec.sparse_decode(idx, val, n, out=acc_a, weight=0.25, accumulate=True, tiles=tiles)
    codec.sparse_decode(idx, val, n, out=acc_b, weight=0.25, accumulate=True)
    assert torch.equal(acc_a, acc_b)


def test_stacked_tiled_and_untiled_decode_agree():
    codec = _codec()
    g = np.random.default_rng(9)
    n, k = 3_000_017, 30_000
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    x[1_000_000:1_050_000] *= 100  # dense tiles (more than 64 entries per tile)
    xd = torch.from_numpy(x).to(DEV)
    pkt = codec.stacked_encode(xd, k, 127, seed=4, counter=2)
    plain = codec.StackedPacket(pkt.idx, pkt.codes, pkt.norm, pkt.n, pkt.levels, None)
    assert torch.equal(codec.stacked_decode(pkt), codec.stacked_decode(plain))
    acc_a = torch.full((n,), -1.0, device=DEV)
    acc_b = acc_a.clone()
    codec.stacked_decode(pkt, out=acc_a, weight=0.5, accumulate=True)
    codec.stacked_decode(plain, out=acc_b, weight=0.5, accumulate=True)
    assert torch.equal(acc_a, acc_b)


# --------------------------------------------------------------------------------------------- stacked
@pytest.mark.parametrize("n,k,levels", [(4096, 41, 127), (1_000_000, 10_000, 127), (25_000_000, 250_000, 127),
                                        (100_000, 1000, 7)])
def test_stacked_philox_matches_oracle(n, k, levels):
    codec = _codec()
    g = np.random.default_rng(n)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    pkt = codec.stacked_encode(xd, k, levels, seed=99, counter=5)
    out = codec.stacked_decode(pkt).cpu().numpy()
    u_all = ref.philox_uniforms(n, 99, 5)
    exp_out, exp_idx, exp_codes, pn = ref.stacked(x, k, levels, lambda idx: u_all[idx])
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), exp_codes)
    assert pkt.norm.item() == pn
    assert gc.same_bits(out, exp_out)


def test_stacked_full_size_1gib_properties():
    """Config 5 at its real size (268,435,456 fp32 = 1 GiB): size-independent properties."""
    codec = _codec()
    n = 268_435_456
    k = n // 100
    gen = torch.Generator(device=DEV).manual_seed(1234)
    x = torch.randn(n, generator=gen, device=DEV) * 1e-3
    pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
    idx = pkt.idx.to(torch.int64)
    assert idx.numel() == k
    assert bool((idx[1:] > idx[:-1]).all())  # ascending, unique
    kept = x[idx]
    masked = x.clone()
    masked[idx] = -float("inf")
    assert kept.min().item() >= masked.max().item()  # exactly the k largest
    assert pkt.norm.item() == kept.abs().max().item()
    out = codec.stacked_decode(pkt)
    nz = torch.nonzero(out).reshape(-1)
    assert torch.equal(nz, idx[kept != 0])
    # decoded values are the two bracketing levels of |x| / norm (unbiased rounding)
    y = kept.abs() / pkt.norm
    lv = out[idx].abs() / pkt.norm
    assert bool(((lv * 127 - torch.floor(y * 127)).abs() <= 1.0001).all())
    del x, masked, out
    torch.cuda.empty_cache()


def test_stacked_full_size_1gib_vs_oracle():
    """Config 5 at its real size against the oracle, bit for bit: kept set, codes, norm and the decoded 1 GiB vector
    (the oracle's O(n) selection and the Philox uniforms of the kept elements only, so it runs in seconds)."""
    codec = _codec()
    n = 268_435_456
    k = n // 100
    x = (np.random.default_rng(2024).standard_normal(n, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    x[np.random.default_rng(5).integers(0, n, n // 20)] = 0.0  # the "realistic" 5 % exact zeros
    xd = torch.from_numpy(x).to(DEV)
    pkt = codec.stacked_encode(xd, k, 127, seed=9, counter=3)
    out = codec.stacked_decode(pkt).cpu().numpy()
    exp_out, exp_idx, exp_codes, pn = ref.stacked(x, k, 127, lambda i: ref.philox_uniforms_at(i, 9, 3), fast=True)
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), exp_codes)
    assert pkt.norm.item() == float(pn)
    assert gc.same_bits(out, exp_out)
    del xd, pkt
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,frac", [(33_554_439, 0.15), (20_000_011, 0.30)])
def test_encode_hbm_overflow_vs_oracle(n, frac):
    """More candidates per block than its LDS holds (kCap = 16384): the blocks keep the rest in the workspace's HBM
    overflow (g-mode) instead of re-reading x — n = 32 M at k = 15 % (~20 K candidates per block) and 20 M at
    k = 30 % (~24 K).  Top-k and stacked encodes against the oracle, bit for bit."""
    codec = _codec()
    k = int(n * frac)
    x = (np.random.default_rng(31).standard_normal(n, dtype=np.float32) * np.float32(1e-3)).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    idx, val, tiles = codec.topk_encode(xd, k, with_tiles=True)
    exp_idx, exp_val = ref.topk_kept_select(x, k)
    assert np.array_equal(idx.cpu().numpy().astype(np.int64), exp_idx)
    assert gc.same_bits(val.cpu().numpy(), exp_val)
    pkt = codec.stacked_encode(xd, k, 127, seed=4, counter=8)
    _, e_idx, e_codes, pn = ref.stacked(x, k, 127, lambda i: ref.philox_uniforms_at(i, 4, 8), fast=True)
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), e_idx)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), e_codes)
    assert pkt.norm.item() == float(pn)
    del xd, pkt
    torch.cuda.empty_cache()


def test_stacked_encode_two_streams():
    """Selects on two streams at once (each with its own workspace) are serialised by the library's gate
    (first switch drains the device, then an event chain); results equal the single-stream ones."""
    codec = _codec()
    n, k = 3_000_000, 30_000
    gen = torch.Generator(device=DEV).manual_seed(77)
    xs = [torch.randn(n, generator=gen, device=DEV) * 1e-3 for _ in range(4)]
    refs = [codec.stacked_encode(x, k, 127, seed=5, counter=i) for i, x in enumerate(xs)]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = [None] * 8
    for r in range(2):
        for i, x in enumerate(xs):
            with torch.cuda.stream(s1 if (i + r) % 2 == 0 else s2):
                got[4 * r + i] = codec.stacked_encode(x, k, 127, seed=5, counter=i)
    torch.cuda.synchronize()
    for j, p in enumerate(got):
        e = refs[j % 4]
        assert torch.equal(p.idx, e.idx) and torch.equal(p.codes, e.codes) and torch.equal(p.norm, e.norm)
        assert torch.equal(p.tiles, e.tiles)


def test_stacked_encode_repeated_calls_identical():
    """Back-to-back encodes of one delta through one workspace (state carried from call to call: epochs,
    histogram zeroing, precomputed Philox words) give identical packets and decodes."""
    codec = _codec()
    n, k = 40_000_000 + 4099, 400_000
    gen = torch.Generator(device=DEV).manual_seed(99)
    x = torch.randn(n, generator=gen, device=DEV) * 1e-3
    ref = codec.stacked_encode(x, k, 127, seed=3, counter=7)
    ref_out = codec.stacked_decode(ref).clone()
    for _ in range(6):
        p = codec.stacked_encode(x, k, 127, seed=3, counter=7)
        assert torch.equal(p.idx, ref.idx) and torch.equal(p.codes, ref.codes) and torch.equal(p.norm, ref.norm)
        assert torch.equal(p.tiles, ref.tiles)
        assert torch.equal(codec.stacked_decode(p), ref_out)
    idx, val, tiles = codec.topk_encode(x, k, with_tiles=True)
    for _ in range(3):
        i2, v2, t2 = codec.topk_encode(x, k, with_tiles=True)
        assert torch.equal(i2, idx) and torch.equal(v2, val) and torch.equal(t2, tiles)


def test_host_pipeline_matches_sequential():
    """HostCodecPipeline (f3): pinned host deltas through H2D / codec / D2H on three streams give exactly the
    sequential path's decoded vectors."""
    from fl_sim_amd.host import HostCodecPipeline

    codec = _codec()
    n, k, m = 1_000_003, 10_000, 5
    gen = torch.Generator(device="cpu").manual_seed(5)
    hx = [(torch.randn(n, generator=gen) * 1e-3).pin_memory() for _ in range(m)]
    hout = [torch.empty(n, dtype=torch.float32).pin_memory() for _ in range(m)]
    pipe = HostCodecPipeline(n, torch.device(DEV))
    sizes = pipe.run(hx, hout, k, 127, seeds=[11] * m, counters=list(range(m)))
    pipe.synchronize()
    for i in range(m):
        pkt = codec.stacked_encode(hx[i].to(DEV), k, 127, seed=11, counter=i)
        ref = codec.stacked_decode(pkt).cpu()
        assert torch.equal(hout[i], ref)
        assert sizes[i] == pkt.nbytes
    with pytest.raises(ValueError):
        pipe.run([torch.empty(n)], [hout[0]], k)  # not pinned


def test_host_wire_pipeline_equals_device_fold():
    """f3 with the packed wire: pinned host deltas -> H2D -> encode -> D2H of the wire only; then the server's H2D of
    each wire -> decode with the client's weight fused into one accumulator.  Equals the device-resident fold of the
    same clients (dist.aggregate_round with the stacked decode-accumulate step) bit for bit; the wires equal the
    device packets."""
    from fl_sim_amd import dist as fdist
    from fl_sim_amd.host import HostWirePipeline

    codec = _codec()
    n, k, m, seed = 3_000_017, 30_000, 5, 21
    gen = torch.Generator(device="cpu").manual_seed(6)
    hx = [(torch.randn(n, generator=gen) * 1e-3).pin_memory() for _ in range(m)]
    w = fdist.sample_weights([100 * (i + 1) for i in range(m)])
    pipe = HostWirePipeline(n, k, 127, torch.device(DEV))
    wires = pipe.new_wires(m)
    pipe.encode(hx, wires, seeds=[seed + i for i in range(m)], counters=[2] * m)
    pipe.synchronize()
    for i in range(m):
        pkt = codec.stacked_encode(hx[i].to(DEV), k, 127, seed=seed + i, counter=2)
        assert torch.equal(wires[i].idx, pkt.idx.cpu()) and torch.equal(wires[i].codes, pkt.codes.cpu())
        assert torch.equal(wires[i].norm, pkt.norm.cpu()) and torch.equal(wires[i].tiles, pkt.tiles.cpu())
        assert wires[i].nbytes == pkt.nbytes
    acc = torch.empty(n, dtype=torch.float32, device=DEV)
    pipe.decode_accumulate(wires, w, acc)
    pipe.wait()
    exp = fdist.aggregate_round([t.to(DEV) for t in hx], w, list(range(m)),
                                fdist.stacked_decode_accumulate(k, seed=seed, counter=2))
    assert torch.equal(acc, exp)


def _adversarial(name):
    """Inputs that drive the encoder off its fast path: a floor that admits too few elements (fallback pass), a
    region with more candidates than a block's LDS (x-mode), and massive ties at the k-th value."""
    if name == "fallback":
        n, S = 4_000_000, 32768
        x = np.full(n, 1e-6, dtype=np.float32)
        x[((np.arange(S) + 0.5) * n / S).astype(np.int64)] = 1.0
        g = np.random.default_rng(2)
        x[g.integers(0, n, 500_000)] = g.random(500_000).astype(np.float32) * 1e-3
        return x, 200_000
    if name == "skewed":
        g = np.random.default_rng(3)
        x = (g.standard_normal(5_000_000) * 1e-4).astype(np.float32)
        x[1_000_000:1_100_000] *= 1000
        return x, 50_000
    g = np.random.default_rng(4)  # ties: a third of the vector holds the k-th value exactly
    x = (g.standard_normal(3_000_000) * 1e-3).astype(np.float32)
    x[g.integers(0, x.size, 1_000_000)] = np.float32(2e-3)
    return x, 30_000


@pytest.mark.parametrize("name", ["fallback", "skewed", "ties"])
def test_stacked_adversarial_matches_oracle_with_tiles(name):
    """The stacked codec off its fast path (fallback pass, x-mode blocks, heavy ties): wire, norm, tile pointers
    and decode equal the oracle's and the index pass's."""
    codec = _codec()
    x, k = _adversarial(name)
    n = x.size
    xd = torch.from_numpy(x).to(DEV)
    pkt = codec.stacked_encode(xd, k, 127, seed=7, counter=3)
    u_all = ref.philox_uniforms(n, 7, 3)
    exp_out, exp_idx, exp_codes, pn = ref.stacked(x, k, 127, lambda idx: u_all[idx])
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), exp_codes)
    assert pkt.norm.item() == pn
    ref_tiles = torch.empty_like(pkt.tiles)
    codec.call("flc_tile_index", codec._p(pkt.idx), k, n, codec._p(ref_tiles), codec._stream(xd.device))
    assert torch.equal(pkt.tiles, ref_tiles)
    assert gc.same_bits(codec.stacked_decode(pkt).cpu().numpy(), exp_out)


def test_stacked_encode_into_reused_packet():
    """stacked_encode(out=packet) overwrites the packet's tensors with the same result as a fresh encode."""
    from fl_sim_amd import codec

    n, k = 1_000_003, 10_000
    g = torch.Generator(device="cuda").manual_seed(77)
    xa = torch.randn(n, generator=g, device="cuda") * 1e-3
    xb = torch.randn(n, generator=g, device="cuda") * 1e-3
    pk = codec.stacked_encode(xa, k, 127, seed=1, counter=1)
    got = codec.stacked_encode(xb, k, 127, seed=2, counter=3, out=pk)
    ref = codec.stacked_encode(xb, k, 127, seed=2, counter=3)
    assert got.idx.data_ptr() == pk.idx.data_ptr()
    assert torch.equal(got.idx, ref.idx) and torch.equal(got.codes[:k], ref.codes[:k])
    assert torch.equal(got.norm, ref.norm) and torch.equal(got.tiles, ref.tiles)
    with pytest.raises(ValueError):
        codec.stacked_encode(xb[:-1], k, 127, out=pk)
