"""Round 4: the headline step with the decode of step i on a second stream, overlapping the encode of step i + 1
(the encode's latency-bound phases leave HBM idle).  Times 20 steps serial (one stream) and overlapped, and checks
that the last decoded output is bit-identical.  Packets of the last two steps are kept alive (the caching allocator
must not hand a packet still being decoded to the next encode)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 28
k = n // 100
dev = torch.device("cuda", 0)
x = torch.randn(n, generator=torch.Generator(device=dev).manual_seed(1234), device=dev) * 1e-3
out = torch.empty(n, device=dev)
s_enc = torch.cuda.current_stream(dev)
s_dec = torch.cuda.Stream(dev)


def serial(c):
    pkt = codec.stacked_encode(x, k, 127, seed=0, counter=c)
    codec.stacked_decode(pkt, out=out)


keep = []


def overlapped(c):
    pkt = codec.stacked_encode(x, k, 127, seed=0, counter=c)
    ev = torch.cuda.Event()
    ev.record(s_enc)
    with torch.cuda.stream(s_dec):
        s_dec.wait_event(ev)
        codec.stacked_decode(pkt, out=out)
    keep.append(pkt)
    del keep[:-3]


def run(fn, reps=20):
    for c in range(5):
        fn(c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s_enc)
    for c in range(reps):
        fn(100 + c)
    e1.record(s_enc)
    s_enc.wait_stream(s_dec)
    e2 = torch.cuda.Event(enable_timing=True)
    e2.record(s_enc)
    torch.cuda.synchronize()
    return e0.elapsed_time(e2) / reps


for rep in range(3):
    for name, fn in (("serial", serial), ("overlapped", overlapped)):
        ms = run(fn)
        h = hashlib.sha256(out.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"{name}: {ms * 1e3:.1f} us/step, {(8 * n + 10 * k) / ms / 1e6:.0f} GB/s, out sha {h}", flush=True)
