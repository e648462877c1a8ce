"""flc_topk_dense_f64 at 25 M float64 elements, k = 1 %: 10 calls, for `rocprofv3 --kernel-trace --stats`
(the per-kernel split of the sample / floor / filter / digit passes / ties / emit)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
x = torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda", dtype=torch.float64)
for _ in range(10):
    codec.topk_dense_f64(x, n // 100)
torch.cuda.synchronize()
print("ok")
