"""Per-kernel times (live HIP-event probes) of the 1 GiB headline step: stacked encode + decode."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from fl_sim_amd import codec, _lib

def probe(name, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.call("flc_probe_set", name.encode())
    _lib.call("flc_probe_read", None, None)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    t, c = ctypes.c_double(), ctypes.c_int64()
    _lib.call("flc_probe_read", ctypes.byref(t), ctypes.byref(c))
    _lib.call("flc_probe_set", None)
    return t.value / max(c.value, 1) * 1e3

n = int(sys.argv[1]) if len(sys.argv) > 1 else 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(int(os.environ.get("SEED", "1")))) * 1e-3
out = torch.empty_like(x)
enc = lambda: codec.stacked_encode(x, k, 127, 1, 0)
print("filter us", round(probe("topk_filter", enc), 1), "select us", round(probe("stacked_select", enc), 1),
      "fused us", round(probe("stacked_encode", enc), 1), "sample us", round(probe("topk_sample", enc), 1), flush=True)
pkt = enc()
print("stacked_decode us", round(probe("stacked_decode", lambda: codec.stacked_decode(pkt, out=out)), 1), flush=True)
print("tiles in pkt:", pkt.tiles is not None, flush=True)
def step():
    p = codec.stacked_encode(x, k, 127, 1, 0)
    codec.stacked_decode(p, out=out)
for _ in range(3):
    step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    step()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"step ms {ms:.4f}  GB/s {(8 * n + 10 * k) / ms / 1e6:.0f}", flush=True)
ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
st = ws[:16 * 8].cpu().numpy().view(np.uint64)
print("state call,err,C,fb,T,maxkey,rounds,t_lo,t_hi,need,ties,strict,path:", [int(v) for v in st[:13]])
