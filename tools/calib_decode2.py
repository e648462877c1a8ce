"""Time decode variants (FLC_DECODE_VARIANT) x grid sizes (FLC_DECODE_BLOCKS) on a 1 GiB stacked packet."""
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
    return t.value / max(c.value, 1) * 1e3

n = 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
out = torch.empty_like(x)
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
ref = codec.stacked_decode(pkt).clone()
acc0 = torch.randn(n, device="cuda") 
for v, blocks in [(40, 0)] + [(v, b) for v in sys.argv[1].split(",") for b in sys.argv[2].split(",")]:
    os.environ["FLC_DECODE_VARIANT"] = str(v)
    os.environ["FLC_DECODE_BLOCKS"] = str(blocks)
    us = probe("stacked_decode", lambda: codec.stacked_decode(pkt, out=out))
    ok = torch.equal(out, ref)
    a = acc0.clone()
    codec.stacked_decode(pkt, out=a, weight=0.5, accumulate=True)
    ok_acc = torch.equal(a, acc0 + 0.5 * ref)
    print(f"decode variant {v} blocks {blocks}: {us:7.1f} us  {4 * n / us / 1e3:6.0f} GB/s  exact={ok} acc_exact={ok_acc}",
          flush=True)
