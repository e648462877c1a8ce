"""GPU parity of the float64 codec (f64.hip) against the reference's float64 fixtures and the oracle.

The reference runs every compressor on whatever dtype x has (compressors.py:267-410); on a float64 vector every
step stays float64.  Checked here:
* compat RNG: the drop-in ``Compressor`` on float64 numpy inputs reproduces the reference's own outputs
  (tests/golden/codec_f64.npz) bit for bit, its send statistics, the streams' positions afterwards, and its
  IndexError when a p = 2 norm underflows to 0 under nonzero elements;
* philox RNG: natural compression and both ditherings match the oracle fed the same Philox uniforms and the same
  norm, bit for bit, up to 4 M elements; the device norms (p = inf exact, p = 2 within 4 ulp of the exact one);
* top-k: the dense output equals the oracle's stable-argsort result (highest indices kept among ties) up to 4 M
  elements, with ties, zeros, NaN and signed zeros; float64 device tensors in, float64 device tensors out.
"""

import os
import random

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc
from tests import golden_f64 as g64

pytestmark = pytest.mark.gpu

F64 = g64.load()
ADAPTIVE = {k: v for k, v in F64.items() if k.startswith("adaptive")}
DENSE = {k: v for k, v in F64.items() if k.split("|")[0] not in ("topk", "randk") and k not in ADAPTIVE}
SPARSE = {k: v for k, v in F64.items() if k.split("|")[0] in ("topk", "randk")}
DEV = "cuda"


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
        kind, L, p, fp64 = g64.dense_params(name)
        if kind == "std":
            nc = Compressor("norm")
            nc.makeIdenticalCompressor()
            (c.makeStandardDitheringFP64 if fp64 else c.makeStandardDitheringFP32)(L, nc, p)
        else:
            (c.makeNaturalDitheringFP64 if fp64 else c.makeNaturalDitheringFP32)(L, 100, p)
    return c


@pytest.mark.parametrize("case", sorted(DENSE))
def test_f64_dense_compressor_matches_reference_fixture(case):
    rec = DENSE[case]
    name, _, seed = case.split("|")
    x = g64.case_input(case, rec)
    c = make_compressor(name)
    gc.seed_all(int(seed))
    if "error" in rec:
        with pytest.raises(IndexError) as ei:
            c.compressVector(x)
        assert str(rec["error"]).endswith(str(ei.value))
        return
    out = c.compressVector(x)
    assert isinstance(out, np.ndarray) and out.dtype == np.float64 and out.shape == x.shape
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])
    assert float(c.last_need_to_send_advance) == float(rec["send"])
    assert g64.check_output(rec, out), case


@pytest.mark.parametrize("case", sorted(SPARSE))
def test_f64_sparse_compressor_matches_reference_fixture(case):
    from fl_sim_amd import Compressor

    rec = SPARSE[case]
    parts = case.split("|")
    name, K, seed = parts[0], int(parts[2]), int(parts[-1])
    x = g64.case_input(case, rec)
    c = Compressor()
    (c.makeTopKCompressor if name == "topk" else c.makeRandKCompressor)(K, len(x))
    gc.seed_all(seed)
    out = c.compressVector(x)
    assert out.dtype == np.float64
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])
    assert float(c.last_need_to_send_advance) == float(rec["send"])
    if name == "topk":
        assert g64.topk_valid(x, out, K), case
        exp, _ = ref.topk(x, K)  # the device's tie rule (stable argsort: the highest indices kept)
        assert g64.same_bits(out, exp), case
    else:
        assert g64.check_output(rec, out), case


@pytest.mark.parametrize("case", sorted(ADAPTIVE))
def test_f64_adaptive_compressor_matches_reference_fixture(case):
    from fl_sim_amd import Compressor

    rec = ADAPTIVE[case]
    x = g64.case_input(case, rec)
    c = Compressor()
    c.makeAdaptiveRandomCompressor(len(x))
    gc.seed_all(int(case.split("|")[-1]))
    if "error" in rec:
        with pytest.raises(ValueError) as ei:
            c.compressVector(x)
        assert str(ei.value) == str(rec["error"])
    else:
        out = c.compressVector(x)
        assert out.dtype == np.float64
        assert list(np.flatnonzero(out)) == list(rec["index"])
        assert g64.check_output(rec, out), case
    assert np.random.random_sample() == float(rec["next_np"])
    assert random.random() == float(rec["next_random"])


@pytest.mark.parametrize("D", [1, 8191, 8193, 1_000_003, 9_000_000])
def test_f64_adaptive_matches_oracle(D):
    from fl_sim_amd import codec

    g = np.random.default_rng(D)
    x = g.standard_cauchy(D) * 1e-3
    x[g.random(D) < 0.1] = 0.0
    xd = torch.from_numpy(x).to(DEV)
    assert int(codec.adaptive_prepare(xd).item()) == 0
    for u in (0.0, 0.37, 0.999999):
        out, index = codec.adaptive_select(xd, u)
        exp, _, ind = ref.adaptive_random(x, D, u)
        assert int(index.item()) == ind, (D, u)
        assert g64.same_bits(out.cpu().numpy(), exp)


def _x64(D, seed, zero_frac=0.05, scale=1e-3):
    g = np.random.default_rng(seed)
    x = g.standard_normal(D) * scale
    x[g.random(D) < zero_frac] = 0.0
    return x


@pytest.mark.parametrize("D", [7, 8191, 65537, 4_000_000])
def test_f64_natural_philox_matches_oracle(D):
    from fl_sim_amd import codec

    x = _x64(D, D)
    x[: min(D, 6)] = [2.0**-1074, -(2.0**600), 1e-310, 3.0, -0.0, 0.0][: min(D, 6)]
    xd = torch.from_numpy(x).to(DEV)
    codes, out = codec.natural_f64(xd, seed=11, counter=5, want_codes=True)
    exp, _, _ = ref.natural64(x, ref.philox_stream(11, 5, D))
    assert g64.same_bits(out.cpu().numpy(), exp)
    assert g64.same_bits(codec.natural_decode_f64(codes, D).cpu().numpy(), exp)


@pytest.mark.parametrize("D", [5, 8192, 100_003, 4_000_000])
@pytest.mark.parametrize("kind,L,p", [("std", 8, np.inf), ("std", 3, 2), ("nat", 8, 2), ("nat", 4, np.inf),
                                      ("std", 127, np.inf)])
def test_f64_dithering_philox_matches_oracle(D, kind, L, p):
    from fl_sim_amd import codec
    from fl_sim_amd._lib import FLC_Q_NATURAL_DITHER, FLC_Q_STANDARD_DITHER

    x = _x64(D, D + L)
    xd = torch.from_numpy(x).to(DEV)
    norm = codec.quant_norm_f64(xd, p)
    pn = np.float64(norm.item())
    if np.isinf(p):
        assert pn == np.max(np.abs(x))  # exact
    else:
        exact = np.sqrt(np.sum(x.astype(np.longdouble) ** 2))
        assert abs(pn - float(exact)) <= 4 * np.spacing(pn)
    k = FLC_Q_STANDARD_DITHER if kind == "std" else FLC_Q_NATURAL_DITHER
    codes, out, nnz = codec.quant_f64(xd, k, L, norm, seed=3, counter=9, want_codes=True, want_nnz=True)
    levels = ref.standard_levels(L) if kind == "std" else ref.natural_levels(L)
    exp, nz, _, _ = ref.dither64(x, levels, pn, ref.philox_stream(3, 9, D))
    assert g64.same_bits(out.cpu().numpy(), exp)
    assert int(nnz.item()) == nz
    dec = codec.quant_decode_f64(codes, D, k, L, norm).cpu().numpy()
    assert g64.same_bits(dec, exp)


# (1 M at 3 % / 5 % / 10 % and 2 M + 1 at 25 %: the band on, the emit from the segments below segcap 1024, from x above)
@pytest.mark.parametrize("D,K", [(10, 3), (4096, 41), (100_003, 1000), (4_000_000, 40_000), (1_000_000, 999_999),
                                 (1_000_000, 30_000), (1_000_000, 50_000), (1_000_000, 100_000), (2_000_001, 500_000)])
def test_f64_topk_matches_oracle(D, K):
    from fl_sim_amd import codec

    x = _x64(D, 7 * D + K)
    exp, _ = ref.topk(x, K)
    got = codec.topk_dense_f64(torch.from_numpy(x).to(DEV), K).cpu().numpy()
    assert g64.same_bits(got, exp)


def test_f64_topk_ties_zeros_nan():
    from fl_sim_amd import codec

    g = np.random.default_rng(5)
    D = 300_001
    x = np.where(g.random(D) < 0.6, 0.0, g.integers(-3, 4, D).astype(np.float64))
    x[g.random(D) < 0.01] = np.nan
    x[g.random(D) < 0.05] = -0.0
    xd = torch.from_numpy(x).to(DEV)
    for K in (1, 2000, 4000, 60_000, 150_000, D - 1):  # tie classes NaN, 3, 2, 1, 0 (with -0)
        exp, _ = ref.topk(x, K)
        got = codec.topk_dense_f64(xd, K).cpu().numpy()
        assert g64.same_bits(got, exp), K


def test_f64_topk_filter_fallbacks():
    """The candidate filter's two ways back to the full passes give the same dense output: a chunk with more
    candidates than its segment (sorted input), and a sample floor that admits fewer than k elements (every sampled
    position 0, every other one -1)."""
    from fl_sim_amd import codec

    n = 1 << 20
    x = np.sort(_x64(n, 4))  # the largest values all in the last chunks
    for K in (n // 100, 12_345):
        exp, _ = ref.topk(x, K)
        assert g64.same_bits(codec.topk_dense_f64(torch.from_numpy(x).to(DEV), K).cpu().numpy(), exp)
    S = 16384  # f64.hip kSample64
    y = np.full(n, -1.0)
    y[((np.arange(S) + 0.5) * n / S).astype(np.int64)] = 0.0  # the sample positions
    # n / 2, S + 5: the floor admits fewer than k; S - 5: the band resolves T = 0 among S ties (tie-index threshold)
    for K in (n // 2, S + 5, S - 5):
        exp, _ = ref.topk(y, K)
        assert g64.same_bits(codec.topk_dense_f64(torch.from_numpy(y).to(DEV), K).cpu().numpy(), exp)
    # the sample's ceiling too low: k + 100 large values, none at a sample position (more than k keys above the band)
    z = y.copy()
    free = np.setdiff1d(np.arange(n), ((np.arange(S) + 0.5) * n / S).astype(np.int64))
    K = 5000
    z[np.random.default_rng(3).choice(free, K + 100, replace=False)] = 5.0
    exp, _ = ref.topk(z, K)
    assert g64.same_bits(codec.topk_dense_f64(torch.from_numpy(z).to(DEV), K).cpu().numpy(), exp)


def test_f64_topk_band_top_bin_past_the_ceiling():
    """The band's top histogram bin can reach past the ceiling t_hi (the band's width need not be a multiple of the
    bin width); the keys above the ceiling were counted apart and must not enter the K-th largest's bin list.  Built
    around the sample (positions (j + 0.5) n / S): at k = 10 % the ceiling's sample rank is 1460 and the floor's 1817
    (f64.hip filt64), so 1459 sampled A = 1.5 + 2^-12, 350 B = 1.5 and 100 C = 0.75 put the ceiling just above B (its
    24-bit key prefix + 1, where A's keys start) and the floor on C: a band 4097 prefix units wide, binned by 4, whose
    top bin holds B (the K-th largest's, 10,000 ties) and A (100,000 keys above the ceiling).  Before the fix the
    list took A's keys too and T came out wrong."""
    from fl_sim_amd import codec

    n, S = 1 << 20, 16384
    spos = ((np.arange(S) + 0.5) * n / S).astype(np.int64)
    g = np.random.default_rng(11)
    x = g.random(n) * 0.1
    A, B, C = 1.5 + 2.0 ** -12, 1.5, 0.75
    x[spos[:1459]] = A
    x[spos[1459:1809]] = B
    x[spos[1809:1909]] = C
    free = g.permutation(np.setdiff1d(np.arange(n), spos))
    na, nb = 100_000 - 1459, 10_000 - 350
    x[free[:na]] = A
    x[free[na:na + nb]] = B
    K = n // 10  # 100,000 A < K <= 110,000 A + B: the K-th largest is a B
    exp, _ = ref.topk(x, K)
    got = codec.topk_dense_f64(torch.from_numpy(x).to(DEV), K).cpu().numpy()
    assert g64.same_bits(got, exp)
    assert sum(codec.topk_status_all().values()) == 0


@pytest.mark.parametrize("K", [150, 1000, 3000])
def test_f64_topk_infinite_kth_value_below_nans(K):
    """Small k (no ceiling from the sample: the NaN keys, the largest, are counted above the band) with the K-th
    largest among +inf ties near the band's top: the NaNs are kept, then the highest-index +infs."""
    from fl_sim_amd import codec

    n = 1 << 20
    g = np.random.default_rng(K)
    x = g.standard_normal(n)
    x[g.choice(n, 100, replace=False)] = np.nan
    free = np.flatnonzero(~np.isnan(x))
    x[g.choice(free, 5000, replace=False)] = np.inf
    exp, _ = ref.topk(x, K)
    got = codec.topk_dense_f64(torch.from_numpy(x).to(DEV), K).cpu().numpy()
    assert g64.same_bits(got, exp)


@pytest.mark.parametrize("n_ties", [3, 5000, 16384, 16385, 100_000])
def test_f64_topk_ties_of_the_kth_value(n_ties):
    """The K-th largest value repeated n_ties times at random positions, k cutting through the ties: the band's bin
    list resolves the highest-index ties itself up to its capacity (16384 keys of the bin), the fallback beyond."""
    from fl_sim_amd import codec

    n = 2_000_003
    g = np.random.default_rng(n_ties)
    x = g.standard_normal(n) * 1e-3
    v = np.sort(x)[-20_000]  # the value at rank 20000 from the top
    pos = g.choice(n, n_ties, replace=False)
    x[pos] = v
    above = int((x > v).sum())
    for K in (above + 1, above + max(1, n_ties // 2), above + n_ties):
        exp, _ = ref.topk(x, K)
        assert g64.same_bits(codec.topk_dense_f64(torch.from_numpy(x).to(DEV), K).cpu().numpy(), exp), K


@pytest.mark.parametrize("n_ties", [100, 400, 1500])
def test_f64_topk_clustered_ties_in_one_chunk(n_ties):
    """Ties of the K-th value packed into one 8192-element chunk at 25 M (12 chunks per select block): 100 ties put more
    of the bin's keys in one block than its 64 list slots (the overflow list); 400 put more band keys in one chunk than
    its LDS slot holds (341: the block's bin keys then come from its segments); 1500 overflow the chunk's segment (the
    band is off, the exact passes run).  k cuts through the ties each time."""
    from fl_sim_amd import codec

    n = 25_000_000
    g = np.random.default_rng(n_ties)
    x = g.standard_normal(n) * 1e-3
    v = np.sort(x)[-(n // 100)]
    c = 1234 * 8192 + 17
    x[c: c + n_ties] = v
    xd = torch.from_numpy(x).to(DEV)
    above = int((x > v).sum())
    for K in (above + n_ties // 3, above + n_ties):
        exp, _ = ref.topk(x, K)
        assert g64.same_bits(codec.topk_dense_f64(xd, K).cpu().numpy(), exp), K
    assert sum(codec.topk_status_all().values()) == 0


def test_f64_topk_full_size_25m():
    """The headline size of the float64 top-k (BASELINE configs[2]'s 25 M, float64): 1 % and 0.1 % against numpy's
    argsort (the oracle), on gaussian and heavy-tailed vectors."""
    from fl_sim_amd import codec

    n = 25_000_000
    g = np.random.default_rng(25)
    for x in (g.standard_normal(n) * 1e-3, g.standard_cauchy(n) * 1e-4):
        xd = torch.from_numpy(x).to(DEV)
        for K in (n // 100, n // 1000):
            exp, _ = ref.topk(x, K)
            assert g64.same_bits(codec.topk_dense_f64(xd, K).cpu().numpy(), exp), K


def test_f64_device_tensor_in_device_tensor_out():
    from fl_sim_amd import Compressor

    x = torch.from_numpy(_x64(50_000, 1)).to(DEV)
    for make in (lambda c: c.makeNaturalCompressorFP64(), lambda c: c.makeTopKCompressor(500, 50_000),
                 lambda c: c.makeNaturalDitheringFP64(4, 50_000, np.inf), lambda c: c.makeIdenticalCompressor()):
        c = Compressor(rng="philox", seed=4)
        make(c)
        out = c.compressVector(x)
        assert out.device.type == "cuda" and out.dtype == torch.float64 and out.shape == x.shape


def test_f64_lazy_and_randk_are_fp64_arithmetic():
    from fl_sim_amd import codec

    x = _x64(10_001, 3, zero_frac=0.0)
    xd = torch.from_numpy(x).to(DEV)
    assert g64.same_bits(codec.scale_div_f64(xd, 0.3).cpu().numpy(), x / 0.3)
    idx = np.random.default_rng(1).permutation(len(x))[:777]
    got = codec.randk_apply_f64(xd, torch.from_numpy(idx.astype(np.int32)), len(x) / 777).cpu().numpy()
    exp, _ = ref.randk(x, 777, len(x), idx)
    assert g64.same_bits(got, exp)
    assert g64.same_bits(codec.copy_f64(xd).cpu().numpy(), x)


def test_f64_edge_shapes_and_views():
    """n = 1, odd n, views at an 8-B (not 16-B) offset, non-contiguous and CPU float64 tensors: same results as the
    oracle / the contiguous aligned input."""
    from fl_sim_amd import Compressor, codec

    base = torch.from_numpy(_x64(20_011, 9)).to(DEV)
    view = base[1:]  # 8-B aligned view: copied once to an aligned buffer
    assert view.data_ptr() % 16 == 8
    for n in (1, 2, 3, 4097):
        x = view[:n]
        exp, _, _ = ref.natural64(x.cpu().numpy(), ref.philox_stream(1, 2, n))
        _, out = codec.natural_f64(x, 1, 2)
        assert g64.same_bits(out.cpu().numpy(), exp), n
        assert g64.same_bits(codec.copy_f64(x).cpu().numpy(), x.cpu().numpy())
    strided = base[::2]
    assert not strided.is_contiguous()
    exp, _ = ref.topk(strided.cpu().numpy(), 100)
    assert g64.same_bits(codec.topk_dense_f64(strided, 100).cpu().numpy(), exp)
    # a CPU float64 tensor goes host -> device -> host and comes back a CPU float64 tensor
    c = Compressor()
    c.makeTopKCompressor(10, 1000)
    xc = torch.from_numpy(_x64(1000, 3))
    out = c.compressVector(xc)
    assert isinstance(out, torch.Tensor) and out.device.type == "cpu" and out.dtype == torch.float64
    exp, _ = ref.topk(xc.numpy(), 10)
    assert g64.same_bits(out.numpy(), exp)


def test_f64_other_dtypes_refused():
    from fl_sim_amd import Compressor

    c = Compressor()
    c.makeIdenticalCompressor()
    with pytest.raises(TypeError):
        c.compressVector(np.arange(10, dtype=np.float16))
    with pytest.raises(TypeError):
        c.compressVector(np.arange(10, dtype=np.int64))


@pytest.mark.parametrize("structured", [False, True])
def test_f64_adaptive_many_special_chunks_vs_oracle(structured):
    """float64: a binade crossing every 24 chunks over ~330 binades — more special chunks in one walk batch than its
    LDS slots (the rest read from memory), still under each scan block's piece limit.  Structured: x doubling exactly
    every 6144 elements makes the running sum land within a few spacings below each power of two, so no special map
    can be validated and those chunks re-run (still exact); with a random factor per element they go through the maps."""
    from tests.test_gpu_adaptive import _crossing_us
    from fl_sim_amd import codec

    n = 2_000_003
    x = np.exp2(np.arange(n) / 6144.0 - 160.0)
    if not structured:
        x *= 1.0 + 0.3 * np.random.default_rng(5).random(n)
    x[1::7] *= -1
    us = _crossing_us(x, limit=64)
    assert len(us) > 100
    xd = torch.from_numpy(x).to(DEV)
    assert int(codec.adaptive_prepare(xd).item()) == 0
    for u in us:
        out, index = codec.adaptive_select(xd, u)
        _, _, ind = ref.adaptive_random(x, n, u)
        assert int(index.item()) == ind, u
    st = codec.adaptive_stats(xd)
    assert st["sequential"] == 0 and st["special"] > 256, st
    if not structured:
        assert st["taken"] >= st["special"] - 8, st


def test_f64_topk_select_timeout_is_reported():
    """a lost co-residency in the grid-synchronised float64 select (Sel64::err) reaches the workspace's
    sticky error word, flc_f64_status reads it (codec.topk_status_all), and with FLC_TOPK_CHECK=1 the call raises.
    FLC_F64_FORCE_TIMEOUT=1 (read once per process: a child) makes the first grid barrier report a timeout."""
    import subprocess
    import sys

    child = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from fl_sim_amd import codec, _lib
x = torch.randn(1 << 20, device="cuda", dtype=torch.float64)
codec.TOPK_CHECK = False
codec.topk_dense_f64(x, 1 << 13)
print("status", max(codec.topk_status_all(reset=True).values()))
codec.TOPK_CHECK = True
try:
    codec.topk_dense_f64(x, 1 << 13)
    print("no error")
except _lib.FlcError as e:
    print("raised", "float64 top-k" in str(e))
print("status", max(codec.topk_status_all(reset=True).values()))
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FLC_F64_FORCE_TIMEOUT="1")
    r = subprocess.run([sys.executable, "-c", child, root], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln and not ln.startswith("/opt")]
    assert lines == ["status 4", "raised True", "status 0"], lines
