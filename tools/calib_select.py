"""Per-kernel times of the stacked encode on 1 GiB under FLC_TOPK_DBG ablations."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec, _lib

def probe(name, fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    _lib.call("flc_probe_set", name.encode()); _lib.call("flc_probe_read", None, None)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    t, c = ctypes.c_double(), ctypes.c_int64()
    _lib.call("flc_probe_read", ctypes.byref(t), ctypes.byref(c)); _lib.call("flc_probe_set", None)
    return t.value / max(c.value, 1) * 1e3

n = 268_435_456; k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
names = ["topk_sample_gather", "topk_sample_select", "topk_filter", "topk_round", "topk_count", "stacked_compact"]
for dbg in (0, 1, 2, 4):
    os.environ["FLC_TOPK_DBG"] = str(dbg)
    codec._WS.clear()
    f = lambda: codec.stacked_encode(x, k, 127, 1, 0)
    res = {nm: round(probe(nm, f), 1) for nm in names}
    print("dbg", dbg, res)
