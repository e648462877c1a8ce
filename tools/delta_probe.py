"""f1: the delta-fused stacked encode (flc_stacked_encode_delta) against the plain encode of the flat delta and the
two-pass (delta_flatten + encode) path, 64 tensors x 2^22 fp32 = 1 GiB."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

nt, per = 64, 1 << 22
g = torch.Generator(device="cuda").manual_seed(3)
loc = [torch.randn(per, generator=g, device="cuda") for _ in range(nt)]
glo = [t + torch.randn(per, generator=g, device="cuda") * 1e-3 for t in loc]
n = nt * per
k = n // 100
flat = codec.delta_flatten(loc, glo)
fns = {
    "plain_encode": lambda: codec.stacked_encode(flat, k, 127, seed=1, counter=2),
    "fused_delta_encode": lambda: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=2),
    "two_pass": lambda: codec.stacked_encode(codec.delta_flatten(loc, glo, out=flat), k, 127, seed=1, counter=2),
}
for name, fn in fns.items():
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    b.synchronize()
    print(f"{name:20s} {a.elapsed_time(b) / 20 * 1e3:8.1f} us")
