"""Timeline of one stacked encode call (diagnostic build, FLC_LIB=diag/lib_stamps.so): the sample kernel's first start
and last end, the encode's block starts and ends (s_memrealtime, 100 MHz), against the host events around the call —
what of the event-timed duration lies outside the kernels' own execution (dispatch, the end-of-kernel cache release).
DELTA=1: the delta-fused encode over 64 tensors.  DECODE=1: the headline step (a decode after each encode)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fl_sim_amd import codec

BLKT_OFF = 175872  # kOffBlkT (topk.hip)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 268_435_456
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1)) * 1e-3
out = torch.empty_like(x)
if os.environ.get("DELTA"):
    gen = torch.Generator(device="cuda").manual_seed(2)
    sizes = [n // 64] * 63 + [n - 63 * (n // 64)]
    glo = [torch.randn(s, device="cuda", generator=gen) for s in sizes]
    loc = [gl + xp for gl, xp in zip(glo, torch.split(x, sizes))]
    encode = lambda it: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=it)
else:
    encode = lambda it: codec.stacked_encode(x, k, 127, 1, it)
dec = bool(os.environ.get("DECODE"))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(8):
    pkt = encode(it)
    if dec:
        codec.stacked_decode(pkt, out=out)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == "topk"][0]
    ws[BLKT_OFF:BLKT_OFF + 1024 * 32].zero_()
    torch.cuda.synchronize()
    if dec:  # the previous packet's decode right before the call, as in the headline step
        codec.stacked_decode(pkt, out=out)
    e0.record()
    pkt = encode(100 + it)
    e1.record()
    torch.cuda.synchronize()
    ev_us = e0.elapsed_time(e1) * 1e3
    bt = ws[BLKT_OFF:BLKT_OFF + 1024 * 32].cpu().numpy().view(np.uint64).astype(np.int64).reshape(1024, 4)
    G = int((bt[256:512, 0] > 0).sum())
    ns = int((bt[512:768, 0] > 0).sum())
    s0, s1 = bt[512:512 + ns, 0].min(), bt[512:512 + ns, 1].max()
    k0 = bt[256:256 + G, 0]
    kend = bt[:G, 3]
    us = lambda a: float(a) * 10 / 1000
    if it < 2:
        continue
    print(f"event {ev_us:6.1f} us | sample {us(s1 - s0):5.1f} | gap sample->encode {us(k0.min() - s1):5.1f} | "
          f"block starts spread {us(k0.max() - k0.min()):4.1f} | encode first start -> last end {us(kend.max() - k0.min()):6.1f} "
          f"| outside the kernels {ev_us - us(kend.max() - s0):5.1f}", flush=True)
