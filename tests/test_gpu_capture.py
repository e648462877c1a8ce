"""Graph capture: the encoders captured in a torch.cuda.CUDAGraph and replayed with changed inputs must
give what the eager calls give on the same inputs, bit for bit.

* configs[1]'s one-launch quantizer (flc_quant_encode_auto): under capture it takes the two-launch path (its exchange
  tag is made on the host per call, so a replay would otherwise meet the previous replay's words);
* the batched stacked encode (flc_stacked_encode_batch) and its delta-fused form: under capture the client table goes
  into the workspace through kernel arguments (fill_table, 2 KB per launch; 48 clients need two chunks), never
  through a recycled host slot."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _capture(fn, stream):
    with torch.cuda.stream(stream):  # warm: workspaces of this stream allocated outside the capture
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        out = fn()
    return g, out


def test_quant_encode_auto_capture_replays_with_new_inputs():
    from fl_sim_amd import codec

    gen = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(10, 417_482, generator=gen, device="cuda") * 1e-3
    s = torch.cuda.Stream()
    g, (pkt, dec) = _capture(lambda: codec.quant_encode_auto(X, 0, 127, seed=4, counter=9), s)
    for r in range(3):
        X.copy_(torch.randn(X.shape, generator=gen, device="cuda") * 10.0 ** (-r - 2))
        X[r, ::7] = 0.0  # (a zero pattern that changes with the replay)
        g.replay()
        torch.cuda.synchronize()
        epk, edec = codec.quant_encode_auto(X.clone(), 0, 127, seed=4, counter=9)
        torch.cuda.synchronize()
        assert torch.equal(pkt.codes, epk.codes) and torch.equal(pkt.norms, epk.norms)
        assert torch.equal(dec.view(torch.int32), edec.view(torch.int32))
    assert codec.quant_status(torch.device("cuda", 0)) == 0


def _fields_equal(a, b, k):
    return (torch.equal(a.idx, b.idx) and torch.equal(a.codes[:k], b.codes[:k]) and torch.equal(a.norm, b.norm)
            and torch.equal(a.tiles, b.tiles))


@pytest.mark.parametrize("delta", [False, True])
def test_batched_stacked_encode_capture_replays_with_new_inputs(delta):
    from fl_sim_amd import codec

    C, n = 48, 20_011
    k = n // 100
    gen = torch.Generator(device="cuda").manual_seed(2 + delta)
    if delta:
        sizes = [4000, 11, 16_000]
        glb = [torch.randn(m, generator=gen, device="cuda") for m in sizes]
        loc = [[t + torch.randn(t.shape, generator=gen, device="cuda") * 1e-3 for t in glb] for _ in range(C)]
        n = sum(sizes)
        k = n // 100
        fn = lambda: codec.stacked_encode_delta_batch(loc, glb, k, 127, seeds=list(range(C)), counter=3)  # noqa: E731
    else:
        xs = [torch.randn(n, generator=gen, device="cuda") * 1e-3 for _ in range(C)]
        fn = lambda: codec.stacked_encode_batch(xs, k, 127, seeds=list(range(C)), counter=3)  # noqa: E731
    s = torch.cuda.Stream()
    g, pks = _capture(fn, s)
    for r in range(3):
        if delta:
            for lp in loc:
                for t in lp:
                    t.add_(torch.randn(t.shape, generator=gen, device="cuda") * 1e-3)
        else:
            for x in xs:
                x.copy_(torch.randn(n, generator=gen, device="cuda") * 1e-3)
        g.replay()
        torch.cuda.synchronize()
        eager = fn()
        torch.cuda.synchronize()
        for c in range(C):
            assert _fields_equal(pks[c], eager[c], k), (r, c)
    assert codec.topk_status(torch.device("cuda", 0)) == 0
