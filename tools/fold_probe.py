"""Time the one-pass wire fold (flc_stacked_fold_wires) against per-client weighted decode-accumulate, 25M x 8."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

n, k, m = 25_000_000, 250_000, int(os.environ.get("M", "8"))
xs = [torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(i)) * 1e-3 for i in range(m)]
stride, _ = codec.stacked_wire_layout(n, k)
recs = torch.empty(m, stride, dtype=torch.uint8, device="cuda")
for i in range(m):
    codec.stacked_encode(xs[i], k, 127, seed=i, counter=1, wire=recs[i])
pk = [codec.wire_packet(recs[i], n, k) for i in range(m)]
w = [0.1 * (i + 1) for i in range(m)]
out = torch.empty(n, device="cuda")


def fold():
    codec.stacked_fold_wires(recs, list(range(m)), w, n, k, out=out)


def dense():
    out.zero_()
    for i in range(m):
        codec.stacked_decode(pk[i], out=out, weight=w[i], accumulate=True)


for name, fn in (("fold", fold), ("dense", dense)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    print(f"{name:6s} {us:8.1f} us  ({4 * n / us / 1e3:.0f} GB/s of output)")
