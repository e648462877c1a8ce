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
