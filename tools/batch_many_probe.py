"""Kernel breakdown of a batched stacked encode of many small clients (run under rocprofv3 --kernel-trace --stats):
C clients x n elements, k = 1 %.  Usage: python tools/batch_many_probe.py C n"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

C = int(sys.argv[1]) if len(sys.argv) > 1 else 100
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
k = n // 100
g = torch.Generator(device="cuda").manual_seed(5)
xs = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(C)]
for _ in range(10):
    codec.stacked_encode_batch(xs, k, 127, seeds=list(range(C)), counter=1)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    codec.stacked_encode_batch(xs, k, 127, seeds=list(range(C)), counter=1)
b.record()
b.synchronize()
print(f"{C} x {n}: {a.elapsed_time(b) / 10 * 1e3:.1f} us per batched encode")
