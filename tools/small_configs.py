"""configs[1] (10 x 417,482 8-bit dithering, batched) and configs[2] (25M top-k 1 %) steps in a loop, for
rocprofv3 --kernel-trace --stats (profiles/r02/*small*).  Prints the per-step times."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(10, 417_482, generator=g, device=dev) * 1e-3
d3, k3 = 25_000_000, 250_000
X3 = torch.randn(d3, generator=g, device=dev) * 1e-3
o3 = torch.empty(d3, device=dev)


def step2(c):
    norms = codec.quant_norm(X)
    pkt = codec.quant_encode(X, 0, 127, norms, seed=0, counter=c, want_nnz=False)
    codec.quant_decode(pkt)


def step2f(c):
    codec.quant_encode_auto(X, 0, 127, seed=0, counter=c)


def step3(c):
    idx, val, tiles = codec.topk_encode(X3, k3, with_tiles=True)
    codec.sparse_decode(idx, val, d3, out=o3, tiles=tiles)


def step2t(c):  # the two-launch form of quant_encode_auto (norm partials, then the encode folding them)
    os.environ["FLC_QUANT_TWO_LAUNCH"] = "1"
    codec.quant_encode_auto(X, 0, 127, seed=0, counter=c)
    del os.environ["FLC_QUANT_TWO_LAUNCH"]


for name, fn, reps in (("config2_quant8_10x417482", step2, 200), ("config2_fused", step2f, 200),
                       ("config2_fused_two_launch", step2t, 200), ("config3_topk1pct_25M", step3, 100)):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    print(name, "us/step", round((time.perf_counter() - t0) * 1e6 / reps, 2))
