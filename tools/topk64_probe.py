"""flc_topk_dense_f64 at 25 M float64 elements, k = 1 %: per-call time with HIP events (20 calls back to back on one
input, then 21 calls rotating over three distinct inputs: 600 MB, not cache-resident), a
check against torch.topk (no ties in a gaussian vector), and 10 more calls for `rocprofv3 --kernel-trace --stats`
(the per-kernel split of sample / filter / gather / fallback / emit)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
k = int(n * float(sys.argv[2]) / 100) if len(sys.argv) > 2 else n // 100  # (argument 2: k in % of n)
x = torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda", dtype=torch.float64)
out = codec.topk_dense_f64(x, k)
exp = torch.zeros_like(x)
idx = torch.topk(x, k).indices
exp[idx] = x[idx]
print("matches torch.topk:", bool(torch.equal(out.view(torch.int64), exp.view(torch.int64))), flush=True)
for _ in range(5):
    codec.topk_dense_f64(x, k)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    e0.record()
    for _ in range(20):
        codec.topk_dense_f64(x, k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"topk_dense_f64 n={n} k={k}: {us:.1f} us/call, {16 * n / us / 1e3:.0f} GB/s of the 16 B/element floor",
          flush=True)
# fresh inputs: three distinct vectors (600 MB, above the 256 MiB memory-side cache) in rotation
xs = [x] + [torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(6 + i), device="cuda",
                        dtype=torch.float64) for i in range(2)]
for i in range(6):
    codec.topk_dense_f64(xs[i % 3], k)
for rep in range(3):
    e0.record()
    for i in range(21):
        codec.topk_dense_f64(xs[i % 3], k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 21
    print(f"topk_dense_f64 n={n} k={k}, 3 inputs rotated: {us:.1f} us/call, {16 * n / us / 1e3:.0f} GB/s", flush=True)
for _ in range(10):
    codec.topk_dense_f64(x, k)
torch.cuda.synchronize()
print("ok")
