"""Time the stacked decode kernel variants (FLC_DECODE_VARIANT) and the filter on a 1 GiB delta."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    return t.value / max(c.value, 1) * 1e3  # us

n = 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
out = torch.empty_like(x)
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
ref = codec.stacked_decode(pkt).clone()
print("filter us", round(probe("topk_filter", lambda: codec.stacked_encode(x, k, 127, 1, 0)), 1))
for v in (10, 11, 20, 21, 40, 41, 80, 81):
    os.environ["FLC_DECODE_VARIANT"] = str(v)
    us = probe("stacked_decode", lambda: codec.stacked_decode(pkt, out=out))
    ok = torch.equal(out, ref)
    print(f"decode variant {v}: {us:7.1f} us  {4 * n / us / 1e3:6.0f} GB/s  exact={ok}")
