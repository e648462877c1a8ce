"""a7 adaptive random at 25M: per-call time of flc_adaptive_prepare + flc_adaptive_select (events around 10 calls),
run under `rocprofv3 --kernel-trace --stats` for the per-kernel split (tools/r03_adaptive.sh)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn(n, generator=g, device=dev, dtype=torch.float64 if os.environ.get("F64") else torch.float32) * 1e-3
for _ in range(3):
    codec.adaptive_prepare(x)
    codec.adaptive_select(x, 0.37)
torch.cuda.synchronize()
for name, fn in (("prepare", lambda: codec.adaptive_prepare(x)), ("select", lambda: codec.adaptive_select(x, 0.37))):
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) * 1e2:.3f} ms per call", flush=True)
t0 = time.perf_counter()
for _ in range(10):
    codec.adaptive_prepare(x)
    _, ind = codec.adaptive_select(x, 0.37)
torch.cuda.synchronize()
print(f"both: {(time.perf_counter() - t0) * 1e2:.3f} ms per call, index {int(ind.item())}", flush=True)
print("walk:", codec.adaptive_stats(x), flush=True)
