"""Host time per headline step (the Python + ctypes + launch work that enqueues one stacked encode + decode), against
the GPU's ≈ 0.39 ms: a step whose host side is slower than its kernels leaves the GPU idle.  Measured as the
enqueue time of 200 steps behind a long-running kernel (so the queue never drains), per variant."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import _lib, codec

D = 268_435_456
K = D // 100
x = torch.randn(D, device="cuda") * 1e-3
out = torch.empty(D, device="cuda")
pk0 = codec.stacked_encode(x, K, 127, seed=0, counter=0)
c = [0]


def plain():
    c[0] += 1
    pk = codec.stacked_encode(x, K, 127, seed=0, counter=c[0])
    codec.stacked_decode(pk, out=out)


def reuse():
    c[0] += 1
    pk = codec.stacked_encode(x, K, 127, seed=0, counter=c[0], out=pk0)
    codec.stacked_decode(pk, out=out)


def size_only():
    _lib.size("flc_topk_workspace_size", D, K)


def empties():
    torch.empty(K, dtype=torch.int32, device="cuda")
    torch.empty(K, dtype=torch.uint8, device="cuda")
    torch.empty(1, dtype=torch.float32, device="cuda")
    torch.empty(D // 1024 + 1, dtype=torch.int32, device="cuda")


variants = {"plain step": plain, "step reusing the packet": reuse, "ws size call": size_only, "4 torch.empty": empties}
for name, fn in variants.items():
    try:
        fn()
    except TypeError as e:
        print(f"{name:28s} skipped ({e})")
        continue
    torch.cuda.synchronize()
    busy = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(40):  # ~ 6 ms of memsets ahead of the enqueued steps
        busy.zero_()
    t0 = time.perf_counter()
    for _ in range(200):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name:28s} host {1e6 * (t1 - t0) / 200:7.1f} us per call", flush=True)
