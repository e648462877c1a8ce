"""Same-box A/B of a run-time switch of the library (an environment variable read once per process, e.g.
FLC_COMPACT_SAMPLE): per-call times of the headline stacked step (1 GiB encode + decode), the stacked encode alone,
the f1 delta-fused encode (1 GiB in 64 tensors), configs[2]'s 25 M top-k step on 8 fresh inputs and a 25 M stacked
encode, in one process.  Run it once per setting, interleaved:
    for v in 1 0 1 0 1 0; do FLC_COMPACT_SAMPLE=$v python tools/env_ab.py FLC_COMPACT_SAMPLE; done
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
D, K = 1 << 28, (1 << 28) // 100
x = torch.randn(D, generator=g, device=dev) * 1e-3
out = torch.empty(D, device=dev)
buf = torch.empty(D, device=dev)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:  # settle (bench.py settle_gpu)
    buf.zero_()
    torch.cuda.synchronize()


def per_call(fn, n, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


ctr = [0]


def step():
    ctr[0] += 1
    codec.stacked_decode(codec.stacked_encode(x, K, 127, seed=0, counter=ctr[0]), out=out)


def enc():
    ctr[0] += 1
    codec.stacked_encode(x, K, 127, seed=0, counter=ctr[0])


res = {v: os.environ.get(v) for v in sys.argv[1:]}
res["step_us"] = round(per_call(step, 40), 1)
res["encode_only_us"] = round(per_call(enc, 40), 1)
del buf
sizes = [(1 << 22) + (i % 3) for i in range(63)]
sizes.append((1 << 28) - sum(sizes))
L = list(torch.split(x, sizes))
G = [torch.randn(n, generator=g, device=dev) for n in sizes]
Lc = [a + b for a, b in zip(L, G)]
res["f1_fused_us"] = round(per_call(lambda: codec.stacked_encode_delta(Lc, G, K, 127, seed=0, counter=1), 10), 1)
del Lc, G, L
d3 = 25_000_000
xs = [torch.randn(d3, generator=g, device=dev) * 1e-3 for _ in range(8)]
o3 = torch.empty(d3, device=dev)
r = [0]


def step3():
    r[0] += 1
    idx, val, tiles = codec.topk_encode(xs[r[0] % 8], d3 // 100, with_tiles=True)
    codec.sparse_decode(idx, val, d3, out=o3, tiles=tiles)


def stacked3():
    r[0] += 1
    codec.stacked_encode(xs[r[0] % 8], d3 // 100, 127, seed=0, counter=r[0])


res["topk25M_fresh_us"] = round(per_call(step3, 40), 1)
res["stacked25M_enc_fresh_us"] = round(per_call(stacked3, 40), 1)
res["topk_err"] = sum(codec.topk_status_all().values())
print(res, flush=True)
