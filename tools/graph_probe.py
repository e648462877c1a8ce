"""Does hipGraph replay (torch.cuda.CUDAGraph) shorten the headline step (sample + encode + decode) or the configs[1]
step?  Eager vs replay of the same calls (fixed seed / counter in the captured graph)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
D = 1 << 28
K = D // 100
x = torch.randn(D, generator=g, device=dev) * 1e-3
out = torch.empty(D, device=dev)
X = torch.randn(10, 417_482, generator=g, device=dev) * 1e-3


def step():
    pkt = codec.stacked_encode(x, K, 127, seed=0, counter=5)
    codec.stacked_decode(pkt, out=out)


def step2():
    codec.quant_encode_auto(X, 0, 127, seed=0, counter=5)


def timeit(fn, reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, fn, reps in (("headline", step, 30), ("config2_fused", step2, 200)):
    e = timeit(fn, reps)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    r = timeit(gr.replay, reps)
    print(f"{name:14s} eager {e:8.1f} us   graph replay {r:8.1f} us")
