"""GPU parity of the client delta formation + flatten (flc_delta_flatten) against the reference
fixture (FedOptClient.communicate run by tests/golden/gen_golden.py) and the oracle, bit for bit: shapes of
config 1, odd and empty tensors, misaligned operands and output slots, and more tensors than one launch carries."""

import numpy as np
import pytest
import torch

from oracle import aggregation_ref as agg_ref
from tests import golden_cases as gc
from tests.golden.gen_golden import CONFIG1_SHAPES, SMALL_SHAPES, delta_inputs

pytestmark = pytest.mark.gpu

AGGV = np.load(f"{gc.GOLDEN}/agg_variants.npz", allow_pickle=False)


def _expected(local, cached):
    return torch.cat([d.reshape(-1) for d in agg_ref.client_delta(local, cached)]).numpy()


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_delta_flatten_matches_reference(tag, shapes):
    from fl_sim_amd import codec

    local, cached = delta_inputs(shapes)
    out = codec.delta_flatten([t.cuda() for t in local], [t.cuda() for t in cached]).cpu().numpy()
    assert gc.sha(out) == str(AGGV[f"delta_{tag}|delta|sha"])


@pytest.mark.parametrize("sizes", [[1], [3, 5, 0, 7, 1], [0], [4, 4, 4], [1_000_003], [4097, 4095, 4096, 8193],
                                   list(range(0, 130))])
def test_delta_flatten_odd_shapes(sizes):
    from fl_sim_amd import codec

    g = torch.Generator().manual_seed(len(sizes))
    cached = [torch.randn(n, generator=g) for n in sizes]
    local = [c + torch.randn(c.shape, generator=g) * 1e-3 for c in cached]
    out = codec.delta_flatten([t.cuda() for t in local], [t.cuda() for t in cached])
    assert out.numel() == sum(sizes)
    assert gc.same_bits(out.cpu().numpy(), _expected(local, cached))


def test_delta_flatten_misaligned_views_and_out():
    from fl_sim_amd import codec

    g = torch.Generator().manual_seed(7)
    base_l = torch.randn(50_001, generator=g).cuda()
    base_g = torch.randn(50_001, generator=g).cuda()
    local = [base_l[1:10_001], base_l[10_003:30_003], base_l[30_004:50_001]]   # not 16-B aligned
    cached = [base_g[2:10_002], base_g[10_000:30_000], base_g[30_004:50_001]]
    total = sum(t.numel() for t in local)
    buf = torch.full((total + 1,), -1.0, device="cuda")
    out = codec.delta_flatten(local, cached, out=buf[1:])                        # out misaligned too
    exp = _expected([t.cpu() for t in local], [t.cpu() for t in cached])
    assert gc.same_bits(out.cpu().numpy(), exp)
    assert buf[0].item() == -1.0


def test_delta_flatten_then_stacked_codec():
    """The client step end to end: delta of a parameter list -> stacked top-k -> 8-bit dither, vs the oracle."""
    from fl_sim_amd import codec
    from oracle import compressors_ref as ref

    local, cached = delta_inputs(CONFIG1_SHAPES)
    flat = codec.delta_flatten([t.cuda() for t in local], [t.cuda() for t in cached])
    n = flat.numel()
    k = n // 100
    pkt = codec.stacked_encode(flat, k, 127, seed=3, counter=9)
    out = codec.stacked_decode(pkt).cpu().numpy()
    x = _expected(local, cached)
    u = ref.philox_uniforms(n, 3, 9)
    exp, exp_idx, _, _ = ref.stacked(x, k, 127, lambda i: u[i])
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx)
    assert gc.same_bits(out, exp)


# ---------------------------------------------------------------------- f1: the delta fused into the encode read
def _same_packet(a, b):
    k = a.idx.numel()
    return (torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k]) and torch.equal(a.norm, b.norm)
            and torch.equal(a.tiles, b.tiles))


def test_stacked_encode_delta_matches_reference_delta_and_oracle():
    """flc_stacked_encode_delta on the config-1 parameter list: the packet of the reference's own delta
    (agg_variants.npz fixture, FedOptClient.communicate) through the oracle's stacked codec, bit for bit."""
    from fl_sim_amd import codec
    from oracle import compressors_ref as ref

    local, cached = delta_inputs(CONFIG1_SHAPES)
    x = _expected(local, cached)
    assert gc.sha(x) == str(AGGV["delta_config1|delta|sha"])
    n = x.size
    k = n // 100
    pkt = codec.stacked_encode_delta([t.cuda() for t in local], [t.cuda() for t in cached], k, 127, seed=3, counter=9)
    exp, exp_idx, exp_codes, pn = ref.stacked(x, k, 127, lambda i: ref.philox_uniforms_at(i, 3, 9), fast=True)
    assert np.array_equal(pkt.idx.cpu().numpy().astype(np.int64), exp_idx)
    assert np.array_equal(pkt.codes[:k].cpu().numpy(), exp_codes) and pkt.norm.item() == float(pn)
    assert gc.same_bits(codec.stacked_decode(pkt).cpu().numpy(), exp)


@pytest.mark.parametrize("sizes", [[1, 7, 3, 100_000, 5], [4097, 4095, 4096, 8193, 0, 16384 * 3 + 1],
                                   [1_000_003], list(range(1, 400)), [16384 * 16 + 3] * 9])
def test_stacked_encode_delta_equals_flatten_then_encode(sizes):
    """Odd sizes (tensor boundaries inside wave steps, not 16-B aligned in the flat space), many tensors, empty
    tensors: the same packet as delta_flatten + stacked_encode."""
    from fl_sim_amd import codec

    g = torch.Generator(device="cuda").manual_seed(len(sizes))
    cached = [torch.randn(n, generator=g, device="cuda") for n in sizes]
    local = [c + torch.randn(c.shape, generator=g, device="cuda") * 1e-3 for c in cached]
    n = sum(sizes)
    k = max(1, n // 100)
    a = codec.stacked_encode_delta(local, cached, k, 127, seed=5, counter=2)
    b = codec.stacked_encode(codec.delta_flatten(local, cached), k, 127, seed=5, counter=2)
    assert _same_packet(a, b)


def test_stacked_encode_delta_misaligned_views():
    from fl_sim_amd import codec

    g = torch.Generator(device="cuda").manual_seed(3)
    base_l = torch.randn(3_000_011, generator=g, device="cuda")
    base_g = torch.randn(3_000_011, generator=g, device="cuda")
    local = [base_l[1:1_000_001], base_l[1_000_003:2_500_003], base_l[2_500_006:3_000_011]]
    cached = [base_g[2:1_000_002], base_g[1_000_000:2_500_000], base_g[2_500_006:3_000_011]]
    n = sum(t.numel() for t in local)
    a = codec.stacked_encode_delta(local, cached, n // 100, 127, seed=1, counter=1)
    b = codec.stacked_encode(codec.delta_flatten(local, cached), n // 100, 127, seed=1, counter=1)
    assert _same_packet(a, b)


def test_stacked_encode_delta_1gib_in_64_tensors():
    """The bench's f1 configuration (1 GiB of parameters in 64 tensors): the same packet as the two-pass path."""
    from fl_sim_amd import codec

    sizes = [(1 << 22) + (i % 3) for i in range(63)]
    sizes.append((1 << 28) - sum(sizes))
    g = torch.Generator(device="cuda").manual_seed(64)
    cached = [torch.randn(n, generator=g, device="cuda") * 0.1 for n in sizes]
    local = [c + torch.randn(c.shape, generator=g, device="cuda") * 1e-3 for c in cached]
    k = (1 << 28) // 100
    a = codec.stacked_encode_delta(local, cached, k, 127, seed=2, counter=6)
    flat = codec.delta_flatten(local, cached)
    b = codec.stacked_encode(flat, k, 127, seed=2, counter=6)
    assert _same_packet(a, b)
    del flat, local, cached
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n_clients,k", [(1, 0), (5, 777), (40, 3000)])
def test_count_nonzero_at_batch_matches_numpy(n_clients, k):
    """flc_count_nonzero_at_batch (the deferred compressed messages' send counts) against numpy: per client the nonzero
    entries of x at k indices, NaN counted, -0.0 not, more clients than one launch takes (32)."""
    import ctypes

    from fl_sim_amd import _lib, codec

    n = 50_001
    g = np.random.default_rng(n_clients + k)
    xs, idxs, exp = [], [], []
    for c in range(n_clients):
        x = np.where(g.random(n) < 0.3, 0.0, g.standard_normal(n)).astype(np.float32)
        x[g.random(n) < 0.01] = np.nan
        x[g.random(n) < 0.05] = -0.0
        idx = np.sort(g.choice(n, k, replace=False)).astype(np.int32)
        xs.append(torch.from_numpy(x).cuda())
        idxs.append(torch.from_numpy(idx).cuda())
        exp.append(int(np.count_nonzero(~(x[idx] == 0.0))))
    counts = [torch.full((1,), -7, dtype=torch.int64, device="cuda") for _ in range(n_clients)]
    P = ctypes.c_void_p * n_clients
    _lib.call("flc_count_nonzero_at_batch", P(*[x.data_ptr() for x in xs]), P(*[i.data_ptr() for i in idxs]),
              n_clients, n, k, P(*[c.data_ptr() for c in counts]), codec._stream(xs[0].device))
    assert [int(c.item()) for c in counts] == exp
