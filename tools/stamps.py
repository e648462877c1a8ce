"""Phase stamps of the persistent select (diagnostic build: make EXTRA=-DFLC_SELECT_STAMPS, block 0 only).

Stamp slots (s_memrealtime, 100 MHz): 0 start, 1 after P0, 2+2r / 3+2r before / after the barrier of
radix round r, 14 / 15 before / after the count barrier, 13 end of compaction.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fl_sim_amd import codec

n = 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
for it in range(5):
    codec.stacked_encode(x, k, 127, 1, it)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
    st = ws[256:256 + 128].cpu().numpy().view(np.uint64).astype(np.int64)
    if it < 2:
        continue
    us = lambda a, b: (st[b] - st[a]) * 10 / 1000  # noqa: E731
    parts = [("P0", 0, 1), ("r0 local", 1, 2), ("r0 barrier", 2, 3)]
    r, last = 1, 3
    while st[2 + 2 * r] > 0 and 2 + 2 * r < 13:
        parts += [(f"r{r} local", last, 2 + 2 * r), (f"r{r} barrier", 2 + 2 * r, 3 + 2 * r)]
        last = 3 + 2 * r
        r += 1
    parts += [("counts", last, 14), ("count barrier", 14, 15), ("compaction", 15, 13)]
    print(" | ".join(f"{nm} {us(a, b):.1f}" for nm, a, b in parts), f"| total {us(0, 13):.1f} us")
