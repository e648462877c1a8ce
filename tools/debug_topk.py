"""Dump the select state of flc_topk_encode (workspace SelState) for a few inputs; compare with numpy.

Diagnostic only (run on the GPU box): `python tools/debug_topk.py`.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fl_sim_amd import codec
from tests import golden_cases as gc

NAMES = "gen lo width shift rem done T need ties strict err C fallback maxkey rounds".split()


def state(ws):
    p = ws[:16].cpu().numpy()
    t_lo = int(p[:4].view(np.uint32)[0])
    t_hi = int(p[8:16].view(np.uint64)[0])
    st = ws[512:512 + 8 * len(NAMES)].cpu().numpy().view(np.uint64)
    d = {a: int(b) for a, b in zip(NAMES, st)}
    d["t_lo"], d["t_hi"] = t_lo, t_hi
    tr = ws[768:768 + 6 * 64].cpu().numpy().view(np.uint64).reshape(6, 8)
    d["trace"] = [[hex(int(v)) if j in (0, 1) else int(v) for j, v in enumerate(row)] for row in tr
                  if row.any()]
    return d


cases = [(7, 3), (100, 1), (4096, 41), (65537, 655), (1 << 20, 10485), (3_000_001, 300_000)]
for n, k in cases:
    g = np.random.default_rng(n + k)
    x = (g.standard_normal(n) * 1e-3).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    idx, val = codec.topk_encode(xd, k)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
    d = state(ws)
    keys = gc.order_keys(x)
    ks = np.sort(keys)
    T = int(ks[n - k])
    print(n, k, {a: (hex(b) if a in ("t_lo", "t_hi", "maxkey", "lo", "T") else b) for a, b in d.items()
                 if a != "trace"})
    for row in d["trace"]:
        print("   round lo width shift rem A digit rem' bincount:", row)
    print("   expect T", hex(T), "count>=t_lo", int((keys >= d["t_lo"]).sum()), "max", hex(int(ks[-1])),
          "strict", int((keys > T).sum()), "ties", int((keys == T).sum()))
    exp = np.sort(np.argsort(keys, kind="stable")[n - k:])
    got = idx.cpu().numpy()
    print("   idx equal", bool(np.array_equal(exp, got)), "first diff",
          int(np.argmax(exp != got)) if not np.array_equal(exp, got) else -1, got[:8], exp[:8])
