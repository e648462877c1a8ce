"""``torch.ops.flcodec.*`` (fl_sim_amd/csrc/torch_ops.cpp): the dispatcher registration of the codec and aggregation
entry points.

CPU: the library loads, every op carries its schema, the Meta kernels infer the output shapes, and a CPU tensor is
refused (no CPU kernel, no fallback).  GPU: each op reproduces the ctypes path (``fl_sim_amd.codec``, itself checked
against the oracle in test_gpu_codec.py) bit for bit, and the stacked op matches the oracle directly.
"""

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc

OPS = {
    "stacked_encode": "flcodec::stacked_encode(Tensor x, int k, int levels=127, int seed=0, int counter=0) -> "
                      "(Tensor idx, Tensor codes, Tensor norm, Tensor tiles)",
    "stacked_decode": "flcodec::stacked_decode(Tensor idx, Tensor codes, Tensor norm, Tensor tiles, int n, "
                      "int levels=127, float weight=1.) -> Tensor",
    "stacked_decode_accumulate_": None,
    "topk_encode": "flcodec::topk_encode(Tensor x, int k) -> (Tensor idx, Tensor val, Tensor tiles)",
    "sparse_decode": None,
    "quant_norm": None,
    "quant_encode": None,
    "quant_decode": None,
    "natural_encode": None,
    "natural_decode": None,
    "weighted_sum_": None,
    "fedopt_step_": None,
    "model_fold_": "flcodec::model_fold_(Tensor(a!)[] dsts, Tensor[] srcs, float[] weights, int init_mode, float beta, "
                   "Tensor(b!)[] theta, Tensor(c!)[] v, int opt=0, float lr=1., float beta2=0., float tau=0.) -> ()",
    "delta_flatten": "flcodec::delta_flatten(Tensor[] theta_local, Tensor[] theta_global) -> Tensor",
    "feddr_combine_": None,
    "stacked_encode_delta": "flcodec::stacked_encode_delta(Tensor[] theta_local, Tensor[] theta_global, int k, "
                            "int levels=127, int seed=0, int counter=0) -> (Tensor idx, Tensor codes, Tensor norm, "
                            "Tensor tiles)",
    "quant_encode_auto": None,
    "adaptive_random": "flcodec::adaptive_random(Tensor x, float u) -> (Tensor out, Tensor index, Tensor status)",
    "stacked_encode_wire": "flcodec::stacked_encode_wire(Tensor x, int k, int levels=127, int seed=0, int counter=0) "
                           "-> Tensor",
    "stacked_fold_wires": None,
    "stacked_encode_batch_wire": "flcodec::stacked_encode_batch_wire(Tensor[] xs, int k, int levels, int[] seeds, "
                                 "int counter=0) -> Tensor",
}


@pytest.fixture(scope="module")
def ops():
    import fl_sim_amd

    fl_sim_amd.load_torch_ops()
    return torch.ops.flcodec


def test_every_op_registered(ops):
    for name, schema in OPS.items():
        op = getattr(ops, name)
        if schema is not None:
            assert str(op.default._schema) == schema


def test_meta_shapes(ops):
    n, k = 100_003, 1000
    x = torch.empty(n, device="meta")
    idx, codes, norm, tiles = ops.stacked_encode(x, k)
    assert (idx.shape, idx.dtype) == ((k,), torch.int32)
    assert (codes.shape, codes.dtype) == ((k,), torch.uint8)
    assert (norm.shape, norm.dtype) == ((1,), torch.float32)
    assert (tiles.shape, tiles.dtype) == (((n + 1023) // 1024 + 1,), torch.int32)
    assert ops.stacked_decode(idx, codes, norm, tiles, n).shape == (n,)
    i2, v2, t2 = ops.topk_encode(x, k)
    assert (v2.shape, v2.dtype, t2.shape) == ((k,), torch.float32, tiles.shape)
    assert ops.sparse_decode(i2, v2, t2, n).shape == (n,)
    x2 = torch.empty(3, 1000, device="meta")
    assert ops.quant_norm(x2, 0).shape == (3,)
    for levels, bits in ((1, 2), (3, 4), (7, 4), (8, 8), (127, 8)):
        c, nnz = ops.quant_encode(x2, torch.empty(3, device="meta"), 0, levels)
        assert c.shape == ((3 * 1000 * bits + 7) // 8,) and nnz.shape == (3,)
    assert ops.quant_decode(c, torch.empty(3, device="meta"), 1000, 0, 127).shape == (3, 1000)
    nc, nz = ops.natural_encode(x)
    assert (nc.shape, nc.dtype, nz.dtype) == ((n,), torch.int16, torch.int64)
    assert ops.natural_decode(nc).shape == (n,)
    ls = [torch.empty(s, device="meta") for s in ((16, 1, 5, 5), (16,), (10, 256))]
    assert ops.delta_flatten(ls, ls).shape == (400 + 16 + 2560,)


def test_cpu_tensors_refused(ops):
    with pytest.raises(NotImplementedError):
        ops.stacked_encode(torch.zeros(64), 4)
    with pytest.raises(NotImplementedError):
        ops.weighted_sum_(torch.zeros(8), [torch.ones(8)], [0.5], 0)
    with pytest.raises(NotImplementedError):
        ops.model_fold_([torch.zeros(8)], [torch.ones(8)], [0.5], 0, 0.0, [], [])


# ------------------------------------------------------------------------------------------------------ GPU parity
def _x(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, generator=g) * 1e-3


def _same(a, b):
    a, b = a.cpu().numpy(), b.cpu().numpy()
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(4096, 41), (417_482, 4174), (1_000_003, 10_000)])
def test_stacked_op_matches_ctypes_and_oracle(ops, n, k):
    from fl_sim_amd import codec

    x = _x(n, n)
    xd = x.cuda()
    idx, codes, norm, tiles = ops.stacked_encode(xd, k, 127, 7, 3)
    pkt = codec.stacked_encode(xd, k, 127, seed=7, counter=3)
    assert _same(idx, pkt.idx) and _same(codes, pkt.codes[:k]) and _same(norm, pkt.norm) and _same(tiles, pkt.tiles)
    out = ops.stacked_decode(idx, codes, norm, tiles, n)
    assert _same(out, codec.stacked_decode(pkt))
    if n <= 417_482:
        u = ref.philox_uniforms(n, 7, 3)
        exp, exp_idx, exp_codes, exp_norm = ref.stacked(x.numpy(), k, 127, lambda i: u[i])
        assert np.array_equal(idx.cpu().numpy().astype(np.int64), exp_idx)
        assert np.array_equal(codes.cpu().numpy(), exp_codes)
        assert gc.same_bits(out.cpu().numpy(), exp)
    acc = torch.full((n,), 0.25, device="cuda")
    r = ops.stacked_decode_accumulate_(acc, idx, codes, norm, tiles, 127, 0.5)
    assert r.data_ptr() == acc.data_ptr()
    exp_acc = torch.full((n,), 0.25, device="cuda")
    codec.stacked_decode(pkt, out=exp_acc, weight=0.5, accumulate=True)
    assert _same(acc, exp_acc)


@pytest.mark.gpu
def test_topk_and_sparse_ops(ops):
    from fl_sim_amd import codec

    n, k = 2_000_000, 20_000
    x = _x(n, 1).cuda()
    idx, val, tiles = ops.topk_encode(x, k)
    e_idx, e_val, e_tiles = codec.topk_encode(x, k, with_tiles=True)
    assert _same(idx, e_idx) and _same(val, e_val) and _same(tiles, e_tiles)
    kept, vals = ref.topk_kept(x.cpu().numpy(), k)
    assert np.array_equal(idx.cpu().numpy().astype(np.int64), kept)
    out = ops.sparse_decode(idx, val, tiles, n, 2.0, 0.5)
    assert _same(out, codec.sparse_decode(e_idx, e_val, n, scale=2.0, weight=0.5, tiles=e_tiles))


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [1, 7, 127])
@pytest.mark.parametrize("p", [0, 2])
def test_quant_ops(ops, levels, p):
    import math

    from fl_sim_amd import codec

    x = _x(4 * 10_001, levels).reshape(4, 10_001).cuda()
    norms = ops.quant_norm(x, p)
    assert _same(norms, codec.quant_norm(x, math.inf if p == 0 else 2))
    codes, nnz = ops.quant_encode(x, norms, 0, levels, 5, 9)
    pkt = codec.quant_encode(x, 0, levels, norms, seed=5, counter=9)
    assert _same(codes, pkt.codes) and _same(nnz, pkt.nnz)
    assert _same(ops.quant_decode(codes, norms, 10_001, 0, levels), codec.quant_decode(pkt))


@pytest.mark.gpu
def test_natural_ops(ops):
    from fl_sim_amd import codec

    x = _x(100_000, 3).cuda()
    x[::7] = 0
    codes, nnz = ops.natural_encode(x, 2, 4)
    e_codes, e_nnz = codec.natural_encode(x, seed=2, counter=4)
    assert _same(codes, e_codes) and _same(nnz, e_nnz)
    assert _same(ops.natural_decode(codes, 0.5), codec.natural_decode(e_codes, x.numel(), weight=0.5))


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [0, 1, 2, 3])
def test_aggregation_ops(ops, opt):
    from fl_sim_amd import codec

    n = 417_482
    srcs = [_x(n, 10 + i).cuda() for i in range(5)]
    w = [float(np.float32(1.0 / (i + 2))) for i in range(5)]
    dst = _x(n, 99).cuda()
    exp = dst.clone()
    r = ops.weighted_sum_(dst, srcs, w, 0, 0.3)
    assert r.data_ptr() == dst.data_ptr()
    codec.weighted_sum(exp, srcs, w, init_mode=0, beta=0.3)
    assert _same(dst, exp)
    theta, v = _x(n, 1).cuda(), _x(n, 2).cuda().abs()
    theta2, v2 = theta.clone(), v.clone()
    name = {0: "avg", 1: "adagrad", 2: "yogi", 3: "adam"}[opt]
    ops.fedopt_step_(theta, dst, v if opt else None, opt, 0.1, 0.99, 1e-3)
    codec.fedopt_step(theta2, dst, v2 if opt else None, name, 0.1, 0.99, 1e-3)
    assert _same(theta, theta2) and _same(v, v2)


@pytest.mark.gpu
def test_ops_run_on_current_stream(ops):
    """Launches follow torch's current stream (no implicit sync): a side-stream encode + decode equals the default."""
    n, k = 1 << 20, 10_000
    x = _x(n, 4).cuda()
    base = ops.stacked_decode(*ops.stacked_encode(x, k, 127, 1, 1), n)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        got = ops.stacked_decode(*ops.stacked_encode(x, k, 127, 1, 1), n)
    torch.cuda.current_stream().wait_stream(s)
    assert _same(got, base)


@pytest.mark.gpu
def test_delta_and_feddr_ops(ops):
    from fl_sim_amd import _lib, codec

    shapes = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (256, 1568), (256,), (10, 256), (10,)]
    g = torch.Generator().manual_seed(3)
    loc = [torch.randn(s, generator=g).cuda() for s in shapes]
    glo = [torch.randn(s, generator=g).cuda() for s in shapes]
    assert _same(ops.delta_flatten(loc, glo), codec.delta_flatten(loc, glo))
    n = 417_482
    th, y, xt = _x(n, 1).cuda(), _x(n, 2).cuda(), _x(n, 3).cuda()
    th2, y2 = th.clone(), y.clone()
    ops.feddr_combine_(th, y, xt, 0.9, 0.91, 0.09, _lib.FLC_PROX_L1, 1e-3)
    codec.feddr_combine(th2, y2, xt, 0.9, 0.91, 0.09, _lib.FLC_PROX_L1, 1e-3)
    assert _same(th, th2) and _same(y, y2)


def test_round2_ops_meta_shapes(ops):
    loc = [torch.empty(100, device="meta"), torch.empty(7, device="meta")]
    idx, codes, norm, tiles = ops.stacked_encode_delta(loc, loc, 10)
    assert idx.shape == (10,) and codes.shape == (10,) and tiles.shape == (2,)
    c, nr, dec = ops.quant_encode_auto(torch.empty(3, 5000, device="meta"), 0, 127)
    assert c.shape == (15000,) and nr.shape == (3,) and dec.shape == (3, 5000)
    out, ind, st = ops.adaptive_random(torch.empty(50, device="meta"), 0.5)
    assert out.shape == (50,) and ind.dtype == torch.int64 and st.dtype == torch.int32


@pytest.mark.gpu
def test_round2_ops_match_codec(ops):
    from fl_sim_amd import codec

    g = torch.Generator(device="cuda").manual_seed(12)
    loc = [torch.randn(n, generator=g, device="cuda") for n in (1000, 3, 50_001)]
    glo = [t + torch.randn(t.shape, generator=g, device="cuda") * 1e-3 for t in loc]
    a = ops.stacked_encode_delta(loc, glo, 510, 127, 3, 4)
    b = codec.stacked_encode_delta(loc, glo, 510, 127, 3, 4)
    assert torch.equal(a[0], b.idx) and torch.equal(a[1], b.codes[:510]) and torch.equal(a[3], b.tiles)
    X = torch.randn(4, 5000, generator=g, device="cuda") * 1e-3
    c, nr, dec = ops.quant_encode_auto(X, 0, 127, 0, 8, 1)
    pkt, dec2 = codec.quant_encode_auto(X, 0, 127, seed=8, counter=1)
    assert torch.equal(c, pkt.codes) and torch.equal(nr, pkt.norms) and torch.equal(dec, dec2)
    x = torch.randn(100_003, generator=g, device="cuda")
    out, ind, st = ops.adaptive_random(x, 0.25)
    exp_out, _, exp_ind = ref.adaptive_random(x.cpu().numpy(), x.numel(), 0.25)
    assert int(st.item()) == 0 and int(ind.item()) == exp_ind and gc.same_bits(out.cpu().numpy(), exp_out)


def test_wire_ops_meta_shapes(ops):
    from fl_sim_amd import codec

    rec = ops.stacked_encode_wire(torch.empty(5000, device="meta"), 50)
    assert rec.shape == (codec.stacked_wire_layout(5000, 50)[0],) and rec.dtype == torch.uint8
    out = ops.stacked_fold_wires(torch.empty(3, rec.numel(), dtype=torch.uint8, device="meta"), [2, 0], [0.5, 0.25],
                                 5000, 50)
    assert out.shape == (5000,) and out.dtype == torch.float32
    recs = ops.stacked_encode_batch_wire([torch.empty(5000, device="meta")] * 4, 50, 127, [1, 2, 3, 4])
    assert recs.shape == (4, rec.numel()) and recs.dtype == torch.uint8


@pytest.mark.gpu
def test_wire_ops_match_codec(ops):
    from fl_sim_amd import codec

    n, k = 300_007, 3_000
    g = torch.Generator(device="cuda").manual_seed(21)
    xs = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(3)]
    recs = torch.stack([ops.stacked_encode_wire(x, k, 127, 5 + i, 2) for i, x in enumerate(xs)])
    stride = recs.shape[1]
    ref_recs = torch.empty(3, stride, dtype=torch.uint8, device="cuda")
    for i, x in enumerate(xs):
        codec.stacked_encode(x, k, 127, seed=5 + i, counter=2, wire=ref_recs[i])
    for i in range(3):  # the payload bytes (padding is never written)
        a, b = codec.wire_packet(recs[i], n, k), codec.wire_packet(ref_recs[i], n, k)
        assert torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k]) and torch.equal(a.tiles, b.tiles)
        assert torch.equal(a.norm, b.norm)
    got = ops.stacked_fold_wires(recs, [1, 2, 0], [0.25, 0.5, 0.125], n, k)
    exp = codec.stacked_fold_wires(ref_recs, [1, 2, 0], [0.25, 0.5, 0.125], n, k)
    assert torch.equal(got.view(torch.int32), exp.view(torch.int32))


@pytest.mark.gpu
def test_batch_wire_op_matches_codec(ops):
    from fl_sim_amd import codec

    n, k = 300_007, 3_000
    g = torch.Generator(device="cuda").manual_seed(22)
    xs = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(5)]
    recs = ops.stacked_encode_batch_wire(xs, k, 127, [9 + i for i in range(5)], 4)
    for i, x in enumerate(xs):
        a = codec.wire_packet(recs[i], n, k)
        b = codec.stacked_encode(x, k, 127, seed=9 + i, counter=4)
        assert torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k]) and torch.equal(a.tiles, b.tiles)
        assert torch.equal(a.norm, b.norm)
