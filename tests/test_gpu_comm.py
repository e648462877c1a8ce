"""The RCCL entries of the C ABI (flc_comm_* / flc_rccl_*, csrc/comm.cpp) on the one GPU a box has: a world of one
(RCCL refuses two ranks on one device, so N > 1 runs only in the driver's multi-GPU bench).  The packed-wire round
composed from the C ABI alone — encode into records, all-gather, one-pass fold — equals dist.aggregate_round_wire and
the dense round bit for bit."""

import numpy as np
import pytest
import torch

from fl_sim_amd import codec, comm
from fl_sim_amd import dist as fdist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world1():
    c = comm.RcclComm(comm.unique_id(), 1, 0, device=0)
    yield c
    c.destroy()


def test_comm_world1_collectives(world1):
    assert world1.size() == (1, 0)
    x = torch.randn(100_003, device="cuda")
    out = torch.empty_like(x)
    world1.reduce(x, out, root=0)
    out2 = torch.empty_like(x)
    world1.allreduce(x, out2)
    b = torch.randint(0, 256, (4099,), dtype=torch.uint8, device="cuda")
    g = torch.empty_like(b)
    world1.allgather(b, g)
    torch.cuda.synchronize()
    assert torch.equal(out, x) and torch.equal(out2, x) and torch.equal(g, b)
    with pytest.raises(ValueError):
        world1.allgather(b, torch.empty(10, dtype=torch.uint8, device="cuda"))


def test_wire_round_through_the_c_abi(world1):
    n, k, n_cl = 1_000_003, 10_000, 4
    w = fdist.sample_weights([100 * (i + 1) for i in range(n_cl)])
    g = torch.Generator(device="cuda").manual_seed(5)
    deltas = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(n_cl)]
    stride, _ = codec.stacked_wire_layout(n, k)
    send = torch.empty(n_cl, stride, dtype=torch.uint8, device="cuda")
    for i, d in enumerate(deltas):
        codec.stacked_encode(d, k, 127, seed=3 + i, counter=1, wire=send[i])
    recv = torch.empty_like(send)
    world1.allgather(send.reshape(-1), recv.reshape(-1))
    got = codec.stacked_fold_wires(recv, list(range(n_cl)), w, n, k)
    exp = fdist.aggregate_round_wire(deltas, w, n_cl, fdist.StackedWireCodec(n, k, seed=3, counter=1))
    dense = fdist.aggregate_round(deltas, w, list(range(n_cl)), fdist.stacked_decode_accumulate(k, seed=3, counter=1))
    bits = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
    assert np.array_equal(bits(got), bits(exp)) and np.array_equal(bits(got), bits(dense))
