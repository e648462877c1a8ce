"""Time tiled decode variants (FLC_DECODE_TILED) on a 1 GiB stacked packet, check exactness, plus a ragged n."""
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

variants = sys.argv[1].split(",")
small = []
for n in (1000, 4099, 70001):
    xs = torch.randn(n, device="cuda") * 1e-3
    ks = max(1, n // 37)
    p = codec.stacked_encode(xs, ks, 127, seed=3, counter=0)
    os.environ["FLC_DECODE_TILED"] = "302"
    small.append((p, codec.stacked_decode(p).clone(), torch.randn(n, device="cuda")))
n = 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
out = torch.empty_like(x)
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
os.environ["FLC_DECODE_TILED"] = "302"
ref = codec.stacked_decode(pkt).clone()
acc0 = torch.randn(n, device="cuda")
for rnd in range(2):
    for v in variants:
        os.environ["FLC_DECODE_TILED"] = v
        us = probe("stacked_decode", lambda: codec.stacked_decode(pkt, out=out))
        ok = torch.equal(out, ref)
        a = acc0.clone()
        codec.stacked_decode(pkt, out=a, weight=0.5, accumulate=True)
        ok_acc = torch.equal(a, acc0 + 0.5 * ref)
        ok_small = all(torch.equal(codec.stacked_decode(p), r) and
                       torch.equal(codec.stacked_decode(p, out=a0.clone(), weight=0.5, accumulate=True), a0 + 0.5 * r)
                       for p, r, a0 in small)
        print(f"tiled decode {v}: {us:7.1f} us  {4 * n / us / 1e3:6.0f} GB/s  exact={ok} acc_exact={ok_acc} "
              f"small={ok_small}", flush=True)
