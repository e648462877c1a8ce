"""Per-step times of the headline step in a fresh process: is the slow start count-based or time-based?
mode: plain | busy (200 ms of memsets first) | sleep (0.2 s idle first)"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
dev = torch.device("cuda", 0)
D, K = 268435456, 2684354
g = torch.Generator(device=dev).manual_seed(1234)
x = torch.randn(D, generator=g, device=dev) * 1e-3
out = torch.empty(D, device=dev)
torch.cuda.synchronize()
if mode == "busy":
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        out.zero_(); torch.cuda.synchronize()
elif mode == "sleep":
    time.sleep(0.2)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(60)]
t0 = time.perf_counter()
for i in range(60):
    ev[i][0].record()
    pkt = codec.stacked_encode(x, K, 127, seed=0, counter=i)
    codec.stacked_decode(pkt, out=out)
    ev[i][1].record()
torch.cuda.synchronize()
ts = [a.elapsed_time(b) * 1e3 for a, b in ev]
print(mode, "first5", [round(t) for t in ts[:5]], "mean 0-4 %.1f 5-24 %.1f 25-59 %.1f" % (
    sum(ts[:5]) / 5, sum(ts[5:25]) / 20, sum(ts[25:]) / 35))
print(mode, "all", [round(t) for t in ts])
