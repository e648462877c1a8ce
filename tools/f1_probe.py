"""The f1 delta-fused stacked encode as tools/env_ab.py times it (1 GiB in 64 tensors, k = 1 %): 30 calls back to
back, for `rocprofv3 --kernel-trace` (tools/ktrace_gaps.py prints each kernel's duration and the idle time before it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
per = (1 << 28) // 64
Lc = [torch.randn(per, generator=g, device=dev) * 1e-3 for _ in range(64)]
G = [torch.randn(per, generator=g, device=dev) * 1e-3 for _ in range(64)]
K = (1 << 28) // 100
for _ in range(5):
    codec.stacked_encode_delta(Lc, G, K, 127, seed=0, counter=1)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(30):
    codec.stacked_encode_delta(Lc, G, K, 127, seed=0, counter=1)
e1.record()
torch.cuda.synchronize()
print(f"f1 stacked_encode_delta: {e0.elapsed_time(e1) * 1e3 / 30:.1f} us per call", flush=True)
