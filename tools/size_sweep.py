"""Stacked encode + decode step time over vector sizes (k = 1 %), up to 2^30 elements (4 GiB): where a block's
candidates outgrow its LDS (x-mode) the encode re-reads its range."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

for lg in (24, 26, 28, 29, 30):
    n = 1 << lg
    k = n // 100
    x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(lg)) * 1e-3
    out = torch.empty(n, device="cuda")

    def step(c):
        pkt = codec.stacked_encode(x, k, 127, seed=0, counter=c)
        codec.stacked_decode(pkt, out=out)

    for c in range(3):
        step(c)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for c in range(5):
        step(c)
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / 5
    err = codec.topk_status(x.device)
    print(f"n=2^{lg} ({4 * n / 2**30:.2f} GiB): {ms:.3f} ms/step, {(8 * n + 10 * k) / ms / 1e6:.0f} GB/s, err {err}",
          flush=True)
    del x, out
    torch.cuda.empty_cache()
