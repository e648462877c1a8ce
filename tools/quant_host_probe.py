"""configs[1]'s one-launch quantizer step (bench.py step2f): host enqueue time per call against the synchronised time
per call and the kernel's event time — is the step host- or GPU-bound?
    python tools/quant_host_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from fl_sim_amd import _lib, codec

dev = torch.device("cuda", 0)
X = torch.randn(10, 417_482, device=dev) * 1e-3
c = [0]


def step():
    c[0] += 1
    codec.quant_encode_auto(X, 0, 127, seed=0, counter=c[0])


for _ in range(50):
    step()
torch.cuda.synchronize()
for n in (10, 30):  # host time of n calls issued back to back (the queue does not fill at these counts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    host = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / n * 1e6
    print(f"{n} calls: host enqueue {host:.1f} us/call, synchronised {tot:.1f} us/call")
# pieces of the host path
t0 = time.perf_counter()
for _ in range(200):
    torch.empty(10 * 417_482, dtype=torch.uint8, device=dev)
print(f"torch.empty: {(time.perf_counter() - t0) / 200 * 1e6:.2f} us")
ws = codec.workspace(dev, codec._ws_size(dev, "flc_quant_workspace_size", 10, 417_482), "quant")
t0 = time.perf_counter()
for _ in range(200):
    codec._stream(dev)
print(f"_stream: {(time.perf_counter() - t0) / 200 * 1e6:.2f} us")
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(50):
    step()
ev[1].record()
torch.cuda.synchronize()
print(f"event time per call (GPU side, back to back): {ev[0].elapsed_time(ev[1]) / 50 * 1e3:.1f} us")
