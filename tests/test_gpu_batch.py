"""GPU parity of the batched stacked encode (flc_stacked_encode_batch): the clients of one round encoded in one
launch, each client's select on its own share of the CUs, equal bit for bit to one single-client encode per client
(stacked_encode, itself pinned against the oracle in test_gpu_codec.py) — plain packets and packed wire records,
more clients than CUs (chunked launches), the take-all sample path, skewed and tied inputs, the HBM overflow
(g-mode) and range re-read (x-mode) paths and NaN, and the configs[3] workload (8 clients x 25M) through the
packed-wire round against the per-client round."""

import pytest
import torch

from fl_sim_amd import codec
from fl_sim_amd import dist as fdist

pytestmark = pytest.mark.gpu


def _x(n, seed, kind="randn"):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(n, generator=g, device="cuda") * 1e-3
    if kind == "zeros":
        x[torch.rand(n, generator=g, device="cuda") < 0.3] = 0.0
    elif kind == "ties":  # few distinct values: the k-th value is tied many times
        x = torch.round(x * 4e3) / 4e3
    elif kind == "skew":
        x[: min(n, 5000)] += 1.0
    return x


def _same(a: codec.StackedPacket, b: codec.StackedPacket, what=""):
    assert torch.equal(a.idx, b.idx), f"idx differ {what}"
    assert torch.equal(a.codes[: a.idx.numel()], b.codes[: b.idx.numel()]), f"codes differ {what}"
    assert torch.equal(a.norm.view(torch.int32), b.norm.view(torch.int32)), f"norm differs {what}"  # (NaN: bits)
    if a.tiles is not None and b.tiles is not None:
        assert torch.equal(a.tiles, b.tiles), f"tiles differ {what}"


@pytest.mark.parametrize("n,k,C", [(70_001, 700, 1), (70_001, 700, 3), (1_000_003, 10_000, 8), (4_194_304, 41_943, 2),
                                   (250_000, 2_500, 17)])
def test_batch_equals_single_encodes(n, k, C):
    kinds = ["randn", "zeros", "ties", "skew"]
    xs = [_x(n, 100 + c, kinds[c % 4]) for c in range(C)]
    seeds = [7 + 3 * c for c in range(C)]
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=seeds, counter=11)
    for c in range(C):
        _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=seeds[c], counter=11), f"client {c}")
    assert codec.topk_status() == 0


def test_batch_more_clients_than_cus():
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    C, n, k = cus + 44, 5_000, 50
    xs = [_x(n, c, "randn" if c % 3 else "ties") for c in range(C)]
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=list(range(C)), counter=2)
    for c in range(0, C, 7):
        _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=c, counter=2), f"client {c}")
    _same(pks[-1], codec.stacked_encode(xs[-1], k, 127, seed=C - 1, counter=2), "last client")


def test_batch_take_all_and_repeat_calls():
    # k close to n: the sample admits everything (take-all path); then the same workspace with other shapes
    for (n, k, C) in [(1_000, 999, 4), (300_001, 3_000, 6), (2_048, 1, 5), (300_001, 3_000, 2)]:
        xs = [_x(n, 7 * c + n % 97) for c in range(C)]
        pks = codec.stacked_encode_batch(xs, k, 127, seeds=[c for c in range(C)], counter=n % 13)
        for c in range(C):
            _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=c, counter=n % 13), f"n={n} client {c}")
    assert codec.topk_status() == 0


def test_batch_into_wire_records_and_fold():
    n, k, C = 2_000_000, 20_000, 5
    xs = [_x(n, 40 + c, "zeros" if c == 2 else "randn") for c in range(C)]
    stride, _ = codec.stacked_wire_layout(n, k)
    recs = torch.zeros(C, stride, dtype=torch.uint8, device="cuda")
    ref = torch.zeros_like(recs)
    codec.stacked_encode_batch(xs, k, 127, seeds=[5 + c for c in range(C)], counter=3, wires=list(recs))
    for c in range(C):
        codec.stacked_encode(xs[c], k, 127, seed=5 + c, counter=3, wire=ref[c])
    for c in range(C):
        _same(codec.wire_packet(recs[c], n, k), codec.wire_packet(ref[c], n, k), f"record {c}")
    w = [0.1 * (c + 1) for c in range(C)]
    a = codec.stacked_fold_wires(recs, list(range(C)), w, n, k, 127)
    b = codec.stacked_fold_wires(ref, list(range(C)), w, n, k, 127)
    assert torch.equal(a, b)


def test_config3_wire_round_batched_equals_per_client():
    # configs[3]: 8 clients x 25M fp32, w_i = ts_i / sum ts with ts_i = 100 (i + 1); one rank owns all 8
    n, k, C = 25_000_000, 250_000, 8
    xs = [_x(n, 300 + c) for c in range(C)]
    w = fdist.sample_weights([100 * (i + 1) for i in range(C)])
    wc = fdist.StackedWireCodec(n, k, 127, seed=0, counter=9)
    got = fdist.aggregate_round_wire(xs, w, C, wc)
    ref = torch.zeros(n, dtype=torch.float32, device="cuda")
    for c in range(C):
        pk = codec.stacked_encode(xs[c], k, 127, seed=c, counter=9)
        codec.stacked_decode(pk, out=ref, weight=float(w[c]), accumulate=True)
    assert torch.equal(got, ref)


def test_batch_overflow_modes_and_nan():
    # g-mode (candidates past a block's LDS kept in the HBM overflow: 15 % kept, ~40 K candidates per block), x-mode
    # (one block's range holds all the large values: more candidates than LDS + overflow, the range re-read) and a NaN
    # (the largest key, always kept) — each in one client of a batch, the other clients plain
    n, k = 32_000_000, 4_800_000
    xs = [_x(n, 500), _x(n, 501, "zeros")]
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=[3, 4], counter=6)
    for c in range(2):
        _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=3 + c, counter=6), f"g-mode client {c}")
    n, k = 2_000_000, 20_000
    xs = [_x(n, 510), _x(n, 511), _x(n, 512)]
    xs[1][:30_000] += 1.0
    xs[2][5] = float("nan")
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=[1, 2, 3], counter=8)
    for c in range(3):
        _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=1 + c, counter=8), f"x-mode/NaN client {c}")
    assert codec.topk_status() == 0


def test_batch_without_tile_pointers():
    n, k, C = 300_001, 3_000, 4
    xs = [_x(n, 600 + c) for c in range(C)]
    pks = codec.stacked_encode_batch(xs, k, 127, seeds=[c for c in range(C)], counter=1, with_tiles=False)
    for c in range(C):
        assert pks[c].tiles is None
        _same(pks[c], codec.stacked_encode(xs[c], k, 127, seed=c, counter=1, with_tiles=False), f"client {c}")
        ref = codec.stacked_decode(codec.stacked_encode(xs[c], k, 127, seed=c, counter=1))
        assert torch.equal(codec.stacked_decode(pks[c]), ref)


def test_delta_batch_equals_single_delta_encodes():
    # a round's clients: each local model = the shared global model + its own update, the delta formed in the pass
    g = torch.Generator(device="cuda").manual_seed(700)
    shapes = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (2048, 123), (123,), (62, 2048), (62,)]
    glob = [torch.randn(*s, generator=g, device="cuda") for s in shapes]
    C = 6
    locs = [[t + torch.randn(*t.shape, generator=g, device="cuda") * 1e-3 for t in glob] for _ in range(C)]
    n = sum(t.numel() for t in glob)
    k = n // 100
    pks = codec.stacked_encode_delta_batch(locs, glob, k, 127, seeds=[10 + c for c in range(C)], counter=4)
    for c in range(C):
        _same(pks[c], codec.stacked_encode_delta(locs[c], glob, k, 127, seed=10 + c, counter=4), f"client {c}")
        _same(pks[c], codec.stacked_encode(codec.delta_flatten(locs[c], glob), k, 127, seed=10 + c, counter=4),
              f"client {c} vs flat")
    # 4-B aligned views (not 16-B) as the tensors
    base = torch.randn(3 * 100_003 + 1, generator=g, device="cuda")
    glob2 = [base[1:100_004], base[100_004:200_007]]
    lbuf = torch.randn(3, 200_010, generator=g, device="cuda")
    locs2 = [[lbuf[c, 3:100_006], lbuf[c, 100_006:200_009]] for c in range(3)]  # 4-B aligned views
    pk2 = codec.stacked_encode_delta_batch(locs2, glob2, 2_000, 127, seeds=[1, 2, 3], counter=2)
    for c in range(3):
        _same(pk2[c], codec.stacked_encode_delta(locs2[c], glob2, 2_000, 127, seed=1 + c, counter=2), f"view {c}")
    assert codec.topk_status() == 0


@pytest.mark.parametrize("with_tiles", [False, True])
def test_topk_batch_equals_single_topk(with_tiles):
    n, k, C = 1_000_003, 10_000, 5
    kinds = ["randn", "zeros", "ties", "skew", "randn"]
    xs = [_x(n, 800 + c, kinds[c]) for c in range(C)]
    got = codec.topk_encode_batch(xs, k, with_tiles=with_tiles)
    for c in range(C):
        ref = codec.topk_encode(xs[c], k, with_tiles=with_tiles)
        assert torch.equal(got[c][0], ref[0]) and torch.equal(got[c][1].view(torch.int32), ref[1].view(torch.int32))
        if with_tiles:
            assert torch.equal(got[c][2], ref[2])
    assert codec.topk_status() == 0


def test_compressor_compress_batch():
    """Compressor.compressBatch: top-k rows through the batched select equal the per-row top-k + decode; the
    dithering batch equals quant_encode_auto of the same batch with the compressor's (seed, counter)."""
    from fl_sim_amd import Compressor

    g = torch.Generator(device="cuda").manual_seed(900)
    X = torch.randn(6, 50_000, generator=g, device="cuda") * 1e-3
    c = Compressor(rng="philox", seed=5)
    c.makeTopKCompressor(500, 50_000)
    got = c.compressBatch(X)
    for r in range(6):
        idx, val, tiles = codec.topk_encode(X[r], 500, with_tiles=True)
        assert torch.equal(got[r], codec.sparse_decode(idx, val, 50_000, tiles=tiles))
    nc = Compressor("norm")
    nc.makeIdenticalCompressor()
    d = Compressor(rng="philox", seed=5)
    d.makeStandardDitheringFP32(8, nc)
    seed, ctr = d.philox.seed, d.philox.counter
    got = d.compressBatch(X)
    assert torch.equal(got, codec.quant_encode_auto(X, 0, d.s, d.p, seed, ctr)[1])


def test_batch_error_word_is_sticky_across_calls():
    """flc_topk_status reports every call since the last reset: a batched call zeroes its headers at the start, but
    not header 0's error word, so an error bit left by an earlier call survives the next batched encode."""
    n, k = 70_001, 700
    xs = [_x(n, 300 + i) for i in range(3)]
    codec.stacked_encode_batch(xs, k, 127, seeds=[1, 2, 3], counter=1)
    assert codec.topk_status(reset=True) == 0
    dev = torch.device("cuda", torch.cuda.current_device())
    ws = codec._WS[(dev.index, codec._stream(dev), "topk_batch")]
    ws[8] = 4  # EncState::err (bytes 8-15 of header 0): an exchange time-out of an "earlier call"
    codec.stacked_encode_batch(xs, k, 127, seeds=[1, 2, 3], counter=2)
    assert codec.topk_status(reset=True) == 4  # still reported after the second call
    codec.stacked_encode_batch(xs, k, 127, seeds=[1, 2, 3], counter=3)
    assert codec.topk_status(reset=True) == 0  # and cleared by the reset
