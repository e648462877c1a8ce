"""How long does the headline step keep speeding up after the onset of load, and which settle removes that?
Each variant runs in a fresh child process (2 s idle between them): settle (kind, seconds), then 400 headline steps
(stacked encode + decode) with per-step events; prints the mean of each group of 25 steps.
kind: memset (bench.py's settle_gpu: out.zero_() + synchronize in a loop) | steps (headline steps, no sync)."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, time, os
sys.path.insert(0, %r)
import torch
from fl_sim_amd import codec
kind, secs = sys.argv[1], float(sys.argv[2])
dev = torch.device("cuda", 0)
D, K = 268435456, 2684354
g = torch.Generator(device=dev).manual_seed(1234)
x = torch.randn(D, generator=g, device=dev) * 1e-3
out = torch.empty(D, device=dev)
torch.cuda.synchronize()
c = [0]
def step():
    c[0] += 1
    pkt = codec.stacked_encode(x, K, 127, seed=0, counter=c[0])
    codec.stacked_decode(pkt, out=out)
t0 = time.perf_counter()
while time.perf_counter() - t0 < secs:
    if kind == "memset":
        out.zero_(); torch.cuda.synchronize()
    else:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
N = 400
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
for i in range(N):
    ev[i][0].record()
    step()
    ev[i][1].record()
torch.cuda.synchronize()
ts = [a.elapsed_time(b) * 1e3 for a, b in ev]
g = [sum(ts[i:i + 25]) / 25 for i in range(0, N, 25)]
print(f"{kind:6s} {secs:4.1f}s  groups of 25: " + " ".join(f"{v:5.1f}" for v in g), flush=True)
""" % ROOT

variants = [("memset", 0.2), ("memset", 1.0), ("steps", 0.2), ("steps", 1.0), ("memset", 0.2), ("steps", 2.0)]
if len(sys.argv) > 1:
    variants = [(a.split(":")[0], float(a.split(":")[1])) for a in sys.argv[1:]]
for kind, secs in variants:
    r = subprocess.run([sys.executable, "-c", CHILD, kind, str(secs)], capture_output=True, text=True, timeout=240)
    print(r.stdout.strip() or r.stderr[-2000:], flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)
    time.sleep(2.0)
