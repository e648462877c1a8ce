"""GPU parity of the packed stacked wire and the one-pass fold of many clients' wires (csrc/wire.hip):
records written by the encoder equal the plain packet bit for bit, and flc_stacked_fold_wires equals the
per-client weighted decode-accumulate chain (the server's sequential fmaf fold) bit for bit —
any client order, more clients than one launch takes, tails, skewed tiles, accumulate into a given vector."""

import numpy as np
import pytest
import torch

from fl_sim_amd import codec
from fl_sim_amd import dist as fdist

pytestmark = pytest.mark.gpu


def _x(n, seed, zeros=False, skew=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, generator=g, device="cuda") * 1e-3
    if zeros:
        x[torch.rand(n, generator=g, device="cuda") < 0.05] = 0.0
    if skew:  # the largest values packed into the first few tiles: > 128 entries per tile over the clients
        x[: min(n, 3000)] += 1.0
    return x


def _records(xs, k, seeds, counter=5):
    n = xs[0].numel()
    stride, _ = codec.stacked_wire_layout(n, k)
    recs = torch.zeros(len(xs), stride, dtype=torch.uint8, device="cuda")
    for i, (x, s) in enumerate(zip(xs, seeds)):
        codec.stacked_encode(x, k, 127, seed=s, counter=counter, wire=recs[i])
    return recs


def _fold_ref(recs, slots, weights, n, k, out):
    for s, w in zip(slots, weights):
        codec.stacked_decode(codec.wire_packet(recs[s], n, k), out=out, weight=float(w), accumulate=True)
    return out


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,k", [(4099, 41), (1_000_003, 10_000)])
def test_encode_into_record_equals_plain_packet(n, k):
    x = _x(n, 1, zeros=True)
    a = codec.stacked_encode(x, k, 127, seed=3, counter=7)
    stride, off = codec.stacked_wire_layout(n, k)
    rec = torch.full((stride,), 0xAB, dtype=torch.uint8, device="cuda")
    b = codec.stacked_encode(x, k, 127, seed=3, counter=7, wire=rec)
    torch.cuda.synchronize()
    assert torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k])
    assert torch.equal(a.norm.view(torch.int32), b.norm.view(torch.int32)) and torch.equal(a.tiles, b.tiles)
    assert b.idx.data_ptr() == rec.data_ptr() + off["idx"]  # views of the record, nothing copied
    out_a = codec.stacked_decode(a)
    out_b = codec.stacked_decode(codec.wire_packet(rec, n, k))
    assert np.array_equal(_bits(out_a), _bits(out_b))


@pytest.mark.parametrize("n,k,m", [(5, 2, 3), (1023, 10, 2), (4099, 41, 1), (4099, 41, 3), (1_000_003, 10_000, 8),
                                   (65_536, 655, 70)])
def test_fold_wires_equals_sequential_decode_accumulate(n, k, m):
    xs = [_x(n, 10 + i, zeros=bool(i % 2)) for i in range(m)]
    recs = _records(xs, k, seeds=list(range(m)))
    g = np.random.default_rng(m)
    slots = list(g.permutation(m))  # any client order
    weights = list(g.random(m) * 0.3 + 0.01)
    exp = _fold_ref(recs, slots, weights, n, k, torch.zeros(n, device="cuda"))
    got = codec.stacked_fold_wires(recs, slots, weights, n, k)
    assert np.array_equal(_bits(got), _bits(exp))
    # accumulating into a given vector (signed zeros included)
    base = torch.randn(n, device="cuda") * 1e-3
    base[::7] = -0.0
    exp2 = _fold_ref(recs, slots, weights, n, k, base.clone())
    got2 = codec.stacked_fold_wires(recs, slots, weights, n, k, out=base.clone(), accumulate=True)
    assert np.array_equal(_bits(got2), _bits(exp2))


def test_fold_wires_skewed_tiles_and_repeated_records():
    n, k, m = 200_003, 2_048, 3
    xs = [_x(n, 40 + i, skew=True) for i in range(m)]
    recs = _records(xs, k, seeds=[5, 6, 7])
    slots, weights = [2, 0, 1, 2], [0.25, -0.5, 1.0, 0.125]  # a record may be folded twice, weights of any sign
    exp = _fold_ref(recs, slots, weights, n, k, torch.zeros(n, device="cuda"))
    got = codec.stacked_fold_wires(recs, slots, weights, n, k)
    assert np.array_equal(_bits(got), _bits(exp))


def test_fold_wires_rejects_bad_arguments():
    n, k = 4099, 41
    recs = _records([_x(n, 1)], k, seeds=[0])
    with pytest.raises(ValueError):
        codec.stacked_fold_wires(recs, [1], [1.0], n, k)  # no record 1
    with pytest.raises(ValueError):
        codec.stacked_fold_wires(recs, [0, 0], [1.0], n, k)
    with pytest.raises(RuntimeError):
        codec.stacked_fold_wires(recs[:, :64].contiguous(), [0], [1.0], n, k)  # stride below the record size


def test_wire_round_world1_equals_dense_round():
    n, k, n_cl = 2_000_000, 20_000, 5
    w = fdist.sample_weights([100 * (i + 1) for i in range(n_cl)])
    deltas = [_x(n, 70 + i, zeros=bool(i % 2)) for i in range(n_cl)]
    dense = fdist.aggregate_round(deltas, w, list(range(n_cl)), fdist.stacked_decode_accumulate(k, seed=9, counter=2))
    wired = fdist.aggregate_round_wire(deltas, w, n_cl, fdist.StackedWireCodec(n, k, seed=9, counter=2))
    assert np.array_equal(_bits(wired), _bits(dense))


def test_fold_wires_nonfinite_weight_takes_every_fma():
    """A non-finite weight turns fmaf(w, +0, acc) into NaN everywhere: the fold must then apply every client's fma to
    every element (the dense variant), like the per-client chain does."""
    n, k = 70_001, 700
    recs = _records([_x(n, 90 + i) for i in range(3)], k, seeds=[1, 2, 3])
    for weights in ([0.5, float("inf"), 0.25], [float("nan"), 1.0, 1.0], [-0.0, 0.0, 2.0]):
        exp = _fold_ref(recs, [0, 1, 2], weights, n, k, torch.zeros(n, device="cuda"))
        got = codec.stacked_fold_wires(recs, [0, 1, 2], weights, n, k)
        assert np.array_equal(_bits(got), _bits(exp))


def test_fold_wires_flat_buffer_equals_2d():
    n, k = 50_001, 500
    recs = _records([_x(n, 60 + i) for i in range(3)], k, seeds=[4, 5, 6])
    a = codec.stacked_fold_wires(recs, [2, 1, 0], [0.5, 0.25, 0.125], n, k)
    b = codec.stacked_fold_wires(recs.reshape(-1), [2, 1, 0], [0.5, 0.25, 0.125], n, k)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_fold_wires_signed_zeros_at_underflow():
    """Near-underflow products: a negative fma result below half the smallest subnormal rounds to -0, which the dense
    chain turns into +0 at the next client with no entry there and a sign-clear weight.  The sparse fold (from +0,
    finite weights) must reproduce that, within one launch and across chained launches (> 64 clients)."""
    n, k = 100_003, 5_000
    a, b, c, d = (_x(n, 120 + i) * 1e-27 for i in range(4))  # kept values ~1.6e-30 .. 4.5e-30 (the largest, > 0)
    xs = [a, b, c, b, c, a, a, d]
    # w * v: 1e-15 -> a nonzero subnormal; +-1e-17 -> +-0.  Elements kept only by b or c end +0 in the chain (the
    # client with w = +1e-17 and no entry there clears their -0) where a sparse fold without that rule keeps -0;
    # elements kept only by d end -0
    weights8 = [1e-15, -1e-17, 1e-17, -1e-17, -2e-17, -1e-17, 1e-17, -1e-17]
    recs = _records(xs, k, seeds=list(range(len(xs))))
    for m in (8, 70):
        slots = [i % 8 for i in range(m)]
        weights = [weights8[i % 8] for i in range(m)]
        exp = _fold_ref(recs, slots, weights, n, k, torch.zeros(n, device="cuda"))
        got = codec.stacked_fold_wires(recs, slots, weights, n, k)
        eb = _bits(exp)
        if m == 8:
            assert (eb == 0x80000000).any()  # the chain does end in -0 somewhere: both cases are exercised
        assert np.array_equal(_bits(got), eb)
