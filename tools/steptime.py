"""Headline step timed three ways on one box: HIP events, perf_counter (bench.py's method), and with the
bench's per-step counter.  Diagnostic for step-time discrepancies."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec

n = 268_435_456; k = n // 100
seed = int(os.environ.get("SEED", "1234"))
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed)) * 1e-3
out = torch.empty_like(x)
ctr = [0]
def step_fixed():
    p = codec.stacked_encode(x, k, 127, 1, 0)
    codec.stacked_decode(p, out=out)
def step_ctr():
    ctr[0] += 1
    p = codec.stacked_encode(x, k, 127, seed=0, counter=ctr[0])
    codec.stacked_decode(p, out=out)
for name, fn in (("fixed", step_fixed), ("ctr", step_ctr), ("fixed", step_fixed), ("ctr", step_ctr)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"{name}: events {e0.elapsed_time(e1) / 20:.4f} ms  wall {(t1 - t0) * 1e3 / 20:.4f} ms", flush=True)
