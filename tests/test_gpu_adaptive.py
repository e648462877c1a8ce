"""GPU parity of the adaptive random compressor (compressors.py:297-301; fl_sim_amd/csrc/adaptive.hip).

* compat mode through the drop-in ``Compressor`` on numpy inputs, against the reference's own outputs
  (tests/golden/codec_sparse.npz adaptive|*, codec_extra.npz: larger, zero-laden and heavy-tailed
  vectors): the same index, the same send statistics, the global streams left where numpy leaves them;
* numpy's errors (NaN / not summing to 1) raised with numpy's message, before any uniform is drawn;
* explicit uniforms against the oracle (numpy's own abs / sum / cumsum / searchsorted) at sizes up to
  25M, with boundary uniforms (0, the smallest, 1 - 2^-53) and adversarial dynamic ranges.
"""

import random

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc

pytestmark = pytest.mark.gpu
DEV = "cuda"
EXTRA = gc.load("codec_extra.npz")


def _compressor(D, rng="compat"):
    from fl_sim_amd import Compressor

    c = Compressor(rng=rng)
    c.makeAdaptiveRandomCompressor(D)
    return c


def _heavy(D, seed):
    """gen_golden.make_heavy."""
    g = np.random.default_rng(20_000 + seed * 104729 + D)
    x = (g.standard_cauchy(D) * 1e-3).astype(np.float32)
    x[g.random(D) < 0.2] = 0.0
    return x


@pytest.mark.parametrize("case", sorted(k for k in EXTRA if not k.startswith("adaptive_err")))
def test_adaptive_matches_reference_fixture(case):
    rec = EXTRA[case]
    kind, D, seed = case.split("|")
    D, seed = int(D), int(seed)
    x = gc.make_input(D, seed, zero_frac=0.05) if kind == "adaptive_z" else _heavy(D, seed)
    assert gc.sha(x) == str(rec["sha_x"])
    c = _compressor(D)
    gc.seed_all(seed)
    out = c.compressVector(x)
    assert np.array_equal(np.flatnonzero(out), rec["index"])
    assert gc.sha(out) == str(rec["sha_out"])
    assert float(c.last_need_to_send_advance) == float(rec["send"]) == 1.0
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


@pytest.mark.parametrize("case", sorted(k for k in EXTRA if k.startswith("adaptive_err")))
def test_adaptive_errors_match_reference(case):
    rec = EXTRA[case]
    x = rec["x"]
    c = _compressor(len(x))
    gc.seed_all(9)
    with pytest.raises(ValueError, match=str(rec["error"])):
        c.compressVector(x)
    assert np.random.random_sample() == float(rec["next_np"])  # nothing drawn
    assert random.random() == float(rec["next_random"])


def test_adaptive_size_mismatch_and_empty():
    c = _compressor(10)
    with pytest.raises(ValueError, match="same size"):
        c.compressVector(np.ones(11, dtype=np.float32))
    from fl_sim_amd import codec

    with pytest.raises(ValueError):
        codec.adaptive_prepare(torch.empty(0, device=DEV))


def _check(x: np.ndarray, us):
    from fl_sim_amd import codec

    xd = torch.from_numpy(x).to(DEV)
    st = int(codec.adaptive_prepare(xd).item())
    assert st == 0
    for u in us:
        out, idx = codec.adaptive_select(xd, u)
        exp_out, _, exp_ind = ref.adaptive_random(x, len(x), u)
        assert int(idx.item()) == exp_ind, (len(x), u)
        o = out.cpu().numpy()
        assert o[exp_ind] == x[exp_ind] and np.count_nonzero(o) == 1


U_EDGES = [0.0, 5e-324, 2.0 ** -53, 0.25, 0.5, 0.7, 1.0 - 2.0 ** -53]


@pytest.mark.parametrize("n", [1, 2, 7, 2047, 2048, 2049, 8191, 8192, 8193, 3 * 8192 + 5, 65_537, 1_000_003])
def test_adaptive_sizes_vs_oracle(n):
    g = np.random.default_rng(n + 1)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    if n > 1:
        x[g.random(n) < 0.05] = 0
        x[0] = 1e-3  # never all zeros
    _check(x, U_EDGES + list(g.random(5)))


@pytest.mark.parametrize("dist", ["cauchy", "lognormal", "spiky", "sparse", "subnormal", "huge"])
def test_adaptive_distributions_vs_oracle(dist):
    n = 2_000_003
    g = np.random.default_rng(7)
    if dist == "cauchy":
        x = g.standard_cauchy(n)
    elif dist == "lognormal":
        x = g.lognormal(0, 8, n) * np.sign(g.standard_normal(n))  # mass spread over many binades
    elif dist == "spiky":
        x = g.standard_normal(n) * 1e-6
        x[g.integers(0, n, 20)] = 1e3
    elif dist == "sparse":
        x = np.zeros(n)
        x[g.integers(0, n, 50)] = g.standard_normal(50)  # long flat stretches of the cdf
    elif dist == "subnormal":
        x = g.standard_normal(n) * 1e-41  # fp32 subnormal inputs
    else:
        x = g.standard_normal(n) * 1e31  # a large fp32 sum (1.6e37)
    x = x.astype(np.float32)
    _check(x, U_EDGES + list(g.random(8)))


def test_adaptive_25M_vs_oracle():
    n = 25_000_000
    g = np.random.default_rng(25)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    x[g.random(n) < 0.05] = 0
    _check(x, [0.0, 0.123456789, 0.5, 0.999999, 1.0 - 2.0 ** -53])


def test_adaptive_philox_mode_is_deterministic():
    g = np.random.default_rng(3)
    x = (g.standard_normal(100_000) * 1e-3).astype(np.float32)
    from fl_sim_amd import Compressor

    outs = []
    for _ in range(2):
        c = Compressor(rng="philox", seed=5)
        c.makeAdaptiveRandomCompressor(len(x))
        outs.append(c.compressVector(torch.from_numpy(x).to(DEV)).cpu().numpy())
    assert np.array_equal(outs[0], outs[1]) and np.count_nonzero(outs[0]) == 1


def test_adaptive_sequential_chain_vs_oracle(monkeypatch):
    """The exact chunk-by-chunk chain the select falls back to when the speculation does not verify, forced."""
    monkeypatch.setenv("FLC_ADAPTIVE_SEQUENTIAL", "1")
    g = np.random.default_rng(11)
    x = (g.standard_normal(1_000_003) * 1e-3).astype(np.float32)
    x[g.random(len(x)) < 0.05] = 0
    _check(x, U_EDGES + list(g.random(4)))


def test_adaptive_binade_every_few_chunks_vs_oracle():
    """Magnitudes doubling every 1000 elements: the running sum crosses a binade every ~4 chunks, more re-run pieces
    than a scan block keeps, so the select takes the sequential chain — still exact."""
    n = 100_000
    x = np.exp2(np.arange(n) / 1000.0).astype(np.float32)
    x[::3] *= -1
    _check(x, U_EDGES + [0.9, 0.99, 0.999])
    from fl_sim_amd import codec

    assert codec.adaptive_stats(torch.from_numpy(x).to(DEV))["sequential"] == 1


def _crossing_us(x: np.ndarray, limit: int = 48):
    """Uniforms on the normalised cdf's own values where the running sum crosses a binade (the special chunks of
    adaptive.hip K3b): the value at the crossing element, one element before it, and the end of its chunk — a cdf one
    ulp off there moves the index."""
    ax = np.abs(x)
    raw = (ax / ax.sum()).astype(np.float64).cumsum()
    cdf = raw / raw[-1]
    e = np.frexp(raw)[1]
    cross = np.flatnonzero(np.diff(e) != 0) + 1
    cross = cross[raw[cross - 1] > 0]
    pick = cross[np.linspace(0, len(cross) - 1, min(limit, len(cross))).astype(int)] if len(cross) else cross
    us = []
    for i in pick:
        end = min(len(x) - 1, (i // 256 + 1) * 256 - 1)
        us += [float(cdf[i]), float(cdf[i - 1]), float(cdf[end])]
    return [u for u in us if 0.0 <= u < 1.0]


def test_adaptive_many_special_chunks_vs_oracle():
    """Magnitudes doubling every 24 chunks: a binade crossing (a special chunk, K3b) every 24 chunks — about 40 per scan
    block, under its piece limit, so they go through the special maps, not the sequential chain.  Uniforms on the cdf's
    values at every sampled crossing."""
    n = 700_001
    x = np.exp2(np.arange(n) / 6144.0 - 60.0).astype(np.float32)
    x[1::5] *= -1
    us = _crossing_us(x)
    assert len(us) > 60
    _check(x, us)
    from fl_sim_amd import codec

    st = codec.adaptive_stats(torch.from_numpy(x).to(DEV))
    assert st["sequential"] == 0 and st["special"] >= 100 and st["taken"] >= st["special"] - 4, st


def test_adaptive_crossing_uniforms_25M_vs_oracle():
    n = 25_000_000
    g = np.random.default_rng(26)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    x[g.random(n) < 0.05] = 0
    _check(x, _crossing_us(x, limit=24))
    from fl_sim_amd import codec

    st = codec.adaptive_stats(torch.from_numpy(x).to(DEV))
    # every binade crossing through a special map: at most a couple of chunks re-run
    assert st["sequential"] == 0 and st["special"] >= 15 and st["reruns"] <= 2, st


@pytest.mark.parametrize("n", [5, 8193, 1_000_003])
def test_adaptive_select_into_unaligned_out(n):
    """The walk's other blocks write the output's zeros: an output view at a 4-B offset is zeroed entirely (head, 16-B
    body, tail) except out[ind] = x[ind]."""
    from fl_sim_amd import codec

    g = np.random.default_rng(n)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    assert int(codec.adaptive_prepare(xd).item()) == 0
    buf = torch.full((n + 2,), 7.0, device=DEV)
    out = buf[1:n + 1]
    _, idx = codec.adaptive_select(xd, 0.4, out=out)
    _, _, exp_ind = ref.adaptive_random(x, n, 0.4)
    assert int(idx.item()) == exp_ind
    o = out.cpu().numpy()
    assert o[exp_ind] == x[exp_ind] and np.count_nonzero(o) == (1 if x[exp_ind] != 0 else 0)
    assert float(buf[0]) == 7.0 and float(buf[n + 1]) == 7.0
