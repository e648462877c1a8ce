"""Does the headline step's time depend on where x (and the output) lie in HBM?  The same 1 GiB delta copied into
several buffers (fresh allocations and views at offsets inside one larger buffer), the headline step (stacked
encode + decode) timed on each, interleaved over three rounds so that drift is not mistaken for placement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

n = 1 << 28
k = n // 100
g = torch.Generator(device="cuda").manual_seed(1234)
x0 = torch.randn(n, generator=g, device="cuda") * 1e-3
out = torch.empty(n, device="cuda")
bufs = {"fresh0": x0}
keep = []
for i in range(1, 3):
    t = torch.empty(n, device="cuda")
    t.copy_(x0)
    bufs[f"fresh{i}"] = t
big = torch.empty(n + (16 << 20), device="cuda")
for off_name, off in [("off4KiB", 1024), ("off64KiB", 16384), ("off2MiB", 1 << 19), ("off6MiB+4KiB", 3 * (1 << 19) + 1024),
                      ("off32MiB", 1 << 23)]:
    v = big[off:off + n]
    bufs[off_name] = v
ctr = [0]


def step(x):
    ctr[0] += 1
    pk = codec.stacked_encode(x, k, 127, seed=1, counter=ctr[0])
    codec.stacked_decode(pk, out=out)


def tm(x, reps=20):
    for _ in range(5):
        step(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        step(x)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


# settle (bench.py's settle_gpu)
for _ in range(100):
    step(x0)
torch.cuda.synchronize()
res = {name: [] for name in bufs}
for r in range(3):
    for name, x in bufs.items():
        if x.data_ptr() != x0.data_ptr() and r == 0:
            x.copy_(x0)
        res[name].append(tm(x))
for name, v in res.items():
    print(f"{name:14s} ptr % 2MiB = {bufs[name].data_ptr() % (1 << 21):8d}  step us: " +
          " ".join(f"{t:6.1f}" for t in v), flush=True)
