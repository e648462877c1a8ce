"""f1: does the delta-fused encode's pass rate depend on where the global parameters lie relative to the local ones?
64 tensors x 2^22 fp32 (1 GiB per operand).  Layouts: the two lists allocated one after the other (global[t] exactly
1 GiB after local[t] in the caching allocator), with a pad between them, and interleaved (local[t], global[t], ...).
Also times delta_flatten (the same two read streams) and the plain encode of the flat delta."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

nt, per = 64, 1 << 22
n = nt * per
k = n // 100


def tm(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def layouts():
    g = torch.Generator(device="cuda").manual_seed(3)
    # (a) consecutive lists
    loc = [torch.randn(per, generator=g, device="cuda") for _ in range(nt)]
    glo = [t + torch.randn(per, generator=g, device="cuda") * 1e-3 for t in loc]
    yield "consecutive", loc, glo
    del loc, glo
    torch.cuda.empty_cache()
    # (b) views of two buffers whose bases differ by 1 GiB + 37 KiB
    big = torch.empty(2 * n + per, device="cuda")
    lb, gb = big[:n], big[n + 9472:2 * n + 9472]
    lb.normal_(generator=g)
    gb.copy_(lb + torch.randn(n, generator=g, device="cuda") * 1e-3)
    yield "offset_37KiB", list(lb.view(nt, per).unbind(0)), list(gb.view(nt, per).unbind(0))
    # (c) interleaved: local[t] then global[t] in one buffer
    il = big[: 2 * n].view(nt, 2, per)
    il[:, 0].normal_(generator=g)
    il[:, 1].copy_(il[:, 0] + torch.randn(nt, per, generator=g, device="cuda") * 1e-3)
    yield "interleaved", list(il[:, 0].unbind(0)), list(il[:, 1].unbind(0))
    # (d) global offset by half a tensor (8 MiB)
    lb, gb = big[:n], big[n + per // 2:2 * n + per // 2]
    lb.normal_(generator=g)
    gb.copy_(lb + torch.randn(n, generator=g, device="cuda") * 1e-3)
    yield "offset_8MiB", list(lb.view(nt, per).unbind(0)), list(gb.view(nt, per).unbind(0))


for name, loc, glo in layouts():
    flat = codec.delta_flatten(loc, glo)
    t_plain = tm(lambda: codec.stacked_encode(flat, k, 127, seed=1, counter=2))
    t_fused = tm(lambda: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=2))
    t_flat = tm(lambda: codec.delta_flatten(loc, glo, out=flat))
    print(f"{name:14s} plain {t_plain:7.1f} us  fused {t_fused:7.1f} us ({t_fused / t_plain:.2f}x)  "
          f"delta_flatten {t_flat:7.1f} us ({12 * n / t_flat / 1e3:.0f} GB/s)", flush=True)
    del flat
