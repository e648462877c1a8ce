"""Read the select kernel's phase stamps (diagnostic build: make EXTRA=-DFLC_SELECT_STAMPS)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from fl_sim_amd import codec
n = 268_435_456; k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
names = ["start", "P0 done", "r0 local", "r0 barrier", "r1 local", "r1 barrier", "r2 local", "r2 barrier", "count local", "count barrier", "compact done"]
for it in range(5):
    pkt = codec.stacked_encode(x, k, 127, 1, it)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
    st = ws[256:256 + 128].cpu().numpy().view(np.uint64)  # stamps follow the 256-B aligned params
    if it < 2: continue
    t = st[:11].astype(np.int64)
    print(" | ".join(f"{names[i]} {(t[i]-t[i-1])*10/1000:.1f}us" for i in range(1, 11) if t[i] > 0), " total", (t[10]-t[0])*10/1000)
