"""The co-residency gate's cost inside a multi-stream process (runtime.cpp Coresident: once persistent launches
have used two streams of a device, every later one waits on and records the gate's event): per-call time of
configs[1]'s one-launch quantizer and configs[2]'s 25 M stacked encode, first in a single-stream process state, then
after one encode on a side stream has switched the gate on.   FLC_LIB=... python tools/gate_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(10, 417_482, generator=g, device=dev) * 1e-3
x25 = torch.randn(25_000_000, generator=g, device=dev) * 1e-3


def per_call(fn, n=200):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 2)


q = lambda i: codec.quant_encode_auto(X, 0, 127, seed=0, counter=i)  # noqa: E731
e = lambda i: codec.stacked_encode(x25, 250_000, 127, seed=0, counter=i)  # noqa: E731
res = {"lib": os.path.basename(os.environ.get("FLC_LIB", "in-tree")), "quant_1stream": per_call(q),
       "enc25M_1stream": per_call(e, 100)}
s = torch.cuda.Stream(dev)
with torch.cuda.stream(s):
    codec.stacked_encode(x25, 250_000, 127, seed=0, counter=1)
torch.cuda.synchronize()
res["quant_gated"] = per_call(q)
res["enc25M_gated"] = per_call(e, 100)
print(res, flush=True)
