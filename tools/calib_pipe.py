"""Stacked encode+decode on 1 GiB deltas: one stream vs two streams (client i+1 encode overlaps client i decode)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec

n = 268_435_456; k = n // 100
dev = torch.device("cuda")
xs = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(i)) * 1e-3 for i in range(3)]
outs = [torch.empty(n, device=dev) for _ in range(3)]
streams = [torch.cuda.Stream() for _ in range(3)]

def run(nstreams, steps):
    for i in range(steps):
        s = streams[i % nstreams]
        with torch.cuda.stream(s):
            pkt = codec.stacked_encode(xs[i % nstreams], k, 127, 1, i)
            codec.stacked_decode(pkt, out=outs[i % nstreams])

for ns in (1, 2, 3, 1, 2, 3):
    run(ns, 4); torch.cuda.synchronize()
    t0 = time.perf_counter(); run(ns, 40); torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 40
    print(f"streams={ns}: {dt*1e6:.1f} us/step  {(8*n+10*k)/dt/1e9:.0f} GB/s")
