"""Dump the top-k select state (workspace params) for a few inputs; compare with numpy."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from fl_sim_amd import codec
from tests import golden_cases as gc

def params(ws):
    b = ws[:128].cpu().numpy().tobytes()
    import struct
    # TopkParams layout: u32 t_lo, u32 fallback, i64 C, u32 maxkey, u32 lo, i32 shift, i32 done, i64 rem,
    # u32 T, u32 err, i64 need, i64 ties_total, i64 strict_total, i64 k
    f = struct.unpack_from("<IIqIIiiqIIqqqq", b)
    names = "t_lo fallback C maxkey lo shift done rem T err need ties strict k".split()
    return dict(zip(names, f))

for n, k in [(65537, 655), (1 << 20, 10485), (300000, 3000)]:
    g = np.random.default_rng(n + k)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    idx, val = codec.topk_encode(xd, k)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
    p = params(ws)
    keys = gc.order_keys(x)
    ks = np.sort(keys)
    T = ks[n - k]
    print(n, k, {a: (hex(b) if a in ("t_lo", "maxkey", "lo", "T") else b) for a, b in p.items()})
    print("   expect T", hex(T), "count>=t_lo", int((keys >= p["t_lo"]).sum()), "max", hex(ks[-1]),
          "strict", int((keys > T).sum()), "ties", int((keys == T).sum()))
    print("   idx nonzero tail", int((idx.cpu().numpy() == 0).sum()))
