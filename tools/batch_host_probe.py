"""Where the batched 100 x 1 M stacked encode's time goes: the GPU-synced time per call against the host's enqueue
time per call (no synchronisation; a host-bound call shows the two equal), and the same for the 10 x 392,313
delta-fused batch."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(77)
xs = [torch.randn(1_000_000, generator=g, device=dev) * 1e-3 for _ in range(100)]
seeds = list(range(100))
fn = lambda: codec.stacked_encode_batch(xs, 10_000, 127, seeds=seeds, counter=1)  # noqa: E731
for _ in range(5):
    fn()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    fn()
torch.cuda.synchronize()
synced = (time.perf_counter() - t0) / 20 * 1e6
t0 = time.perf_counter()
for _ in range(20):
    fn()
host = (time.perf_counter() - t0) / 20 * 1e6
torch.cuda.synchronize()
print(f"stacked 100 x 1M: {synced:.1f} us per call synced, {host:.1f} us host enqueue per call", flush=True)
