"""Per-kernel times (HIP events via the library probe) of the stacked encode + decode on 1 GiB.

Usage (GPU box): python tools/calib_filter.py <label>; used with builds of different
FLC_FILTER_VARIANT / FLC_DECODE_VARIANT values (tools/calib_variants.sh).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import _lib, codec


def probe(name, fn, reps=10):
    for _ in range(2):
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


n = 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
out = torch.empty_like(x)
pkt = codec.stacked_encode(x, k, 127, 1, 0)
enc = lambda: codec.stacked_encode(x, k, 127, 1, 0)  # noqa: E731
dec = lambda: codec.stacked_decode(pkt, out=out)  # noqa: E731
res = {}
for nm in ("topk_sample_gather", "topk_sample_select", "topk_filter", "stacked_select"):
    res[nm] = round(probe(nm, enc), 1)
for nm in ("tile_index", "stacked_decode"):
    res[nm] = round(probe(nm, dec), 1)
res["filter_GBps"] = round(4 * n / res["topk_filter"] / 1e3, 0)
res["decode_GBps"] = round(4 * n / res["stacked_decode"] / 1e3, 0)
print(sys.argv[1] if len(sys.argv) > 1 else "", res, flush=True)
