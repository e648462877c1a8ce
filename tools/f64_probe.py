"""The float64 codec (f64.hip) at 25 M elements: per-call time of each entry point (events around 10 calls), with its
algorithmic bytes and the HBM fraction (8 TB/s), for DESIGN.md §3.6."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402
from fl_sim_amd._lib import FLC_Q_STANDARD_DITHER  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn(n, generator=g, device=dev, dtype=torch.float64) * 1e-3
norm = codec.quant_norm_f64(x, float("inf"))


def tm(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


cases = {  # name: (call, algorithmic bytes)
    "copy_f64": (lambda: codec.copy_f64(x), 16 * n),
    "natural_f64 (encode+decode, philox)": (lambda: codec.natural_f64(x, 1, 2), 16 * n),
    "quant_norm_f64 (p=inf)": (lambda: codec.quant_norm_f64(x, float("inf")), 8 * n),
    "quant_f64 (std s=8, philox, decoded out)": (lambda: codec.quant_f64(x, FLC_Q_STANDARD_DITHER, 8, norm, 1, 2), 16 * n),
    "topk_dense_f64 (k = 1 %)": (lambda: codec.topk_dense_f64(x, n // 100), 16 * n),
}
for name, (fn, b) in cases.items():
    ms = tm(fn)
    print(f"{name:45s} {ms:8.3f} ms  {b / ms / 1e6:8.1f} GB/s  frac {b / ms / 1e6 / 8000:.3f}", flush=True)
