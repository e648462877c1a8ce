"""The weighted, non-accumulating decode (``weight != 1``, ``accumulate=False``: out = fl(weight * decoded), the
client's weight applied on the way out, csrc/sparse.hip) pinned against the oracle (until now only
self-compared, tests/test_torch_ops.py): top-k (idx, val) and stacked wires, tiled and untiled decodes, at tail sizes
that are not multiples of the 1024-output tile, with positive, negative and subnormal-producing weights."""

import numpy as np
import pytest
import torch

from oracle import compressors_ref as ref
from tests import golden_cases as gc

pytestmark = pytest.mark.gpu

F32 = np.float32


def _x(n, seed):
    g = np.random.default_rng(seed)
    x = (g.standard_normal(n) * 1e-3).astype(F32)
    x[g.random(n) < 0.05] = 0.0
    return x


@pytest.mark.parametrize("n", [1_000_003, 4097, 70_001])
@pytest.mark.parametrize("weight", [0.37, -1.5, 3e-39, 1.0])
@pytest.mark.parametrize("tiled", [True, False])
def test_topk_weighted_decode_matches_oracle(n, weight, tiled):
    from fl_sim_amd import codec

    x = _x(n, n + 1)
    k = n // 100
    idx, val, tiles = codec.topk_encode(torch.from_numpy(x).cuda(), k, with_tiles=True)
    out = codec.sparse_decode(idx, val, n, weight=weight, tiles=tiles if tiled else None).cpu().numpy()
    dense, _ = ref.topk(x, k)  # the reference's decoded vector (+0 where not kept)
    exp = (F32(weight) * dense).astype(F32)
    assert gc.same_bits(out, exp)


@pytest.mark.parametrize("n", [1_000_003, 4097, 70_001])
@pytest.mark.parametrize("weight", [0.37, -1.5, 3e-39])
@pytest.mark.parametrize("tiled", [True, False])
def test_stacked_weighted_decode_matches_oracle(n, weight, tiled):
    from fl_sim_amd import codec

    x = _x(n, n + 2)
    k = n // 100
    pkt = codec.stacked_encode(torch.from_numpy(x).cuda(), k, 127, seed=7, counter=3, with_tiles=tiled)
    out = codec.stacked_decode(pkt, weight=weight).cpu().numpy()
    dense, _, _, _ = ref.stacked(x, k, 127, lambda i: ref.philox_uniforms_at(i, 7, 3), fast=True)
    exp = (F32(weight) * dense).astype(F32)
    assert gc.same_bits(out, exp)


@pytest.mark.parametrize("weight", [0.37, -1.5])
def test_wire_record_weighted_decode_matches_oracle(weight):
    """A record of the packed wire (the form a client message carries) decoded with its client's weight."""
    from fl_sim_amd import codec

    n = 1_000_003
    k = n // 100
    x = _x(n, 11)
    stride, _ = codec.stacked_wire_layout(n, k)
    rec = torch.empty(stride, dtype=torch.uint8, device="cuda")
    codec.stacked_encode(torch.from_numpy(x).cuda(), k, 127, seed=2, counter=1, wire=rec)
    out = codec.stacked_decode(codec.wire_packet(rec, n, k), weight=weight).cpu().numpy()
    dense, _, _, _ = ref.stacked(x, k, 127, lambda i: ref.philox_uniforms_at(i, 2, 1), fast=True)
    assert gc.same_bits(out, (F32(weight) * dense).astype(F32))
