"""The batched stacked encode (flc_stacked_encode_batch) against one launch per client, k = 1 %:
configs[3] (8 clients x 25M), 10 clients of cnn_femmist_tiny's delta (417,482; BASELINE configs[1]'s model) and
100 clients of a 1M-parameter delta; and the configs[3] packed-wire round at N = 1 (8 encodes + the fold)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec
from fl_sim_amd import dist as fdist


def tm(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


g = torch.Generator(device="cuda").manual_seed(5)
for n, C in [(25_000_000, 8), (417_482, 10), (1_000_000, 100)]:
    k = n // 100
    xs = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(C)]
    seeds = list(range(C))
    t_b = tm(lambda: codec.stacked_encode_batch(xs, k, 127, seeds=seeds, counter=1))
    t_1 = tm(lambda: [codec.stacked_encode(x, k, 127, seed=s, counter=1) for x, s in zip(xs, seeds)])
    rd = 4 * n * C + 5 * k * C
    print(f"{C:4d} clients x {n:>10,d}: batched {t_b:8.1f} us ({rd / t_b / 1e3:6.0f} GB/s)   one launch per client "
          f"{t_1:8.1f} us ({rd / t_1 / 1e3:6.0f} GB/s)   x{t_1 / t_b:.2f}", flush=True)
    del xs
n, C = 25_000_000, 8
k = n // 100
xs = [torch.randn(n, generator=g, device="cuda") * 1e-3 for _ in range(C)]
w = fdist.sample_weights([100 * (i + 1) for i in range(C)])
wc = fdist.StackedWireCodec(n, k, 127)
out = torch.empty(n, device="cuda")


class OneByOne:
    stride, n = wc.stride, wc.n
    encode_into, fold = wc.encode_into, wc.fold


t_r = tm(lambda: fdist.aggregate_round_wire(xs, w, C, wc, out=out))
t_r1 = tm(lambda: fdist.aggregate_round_wire(xs, w, C, OneByOne, out=out))
print(f"configs[3] wire round at N = 1: batched encode {t_r:8.1f} us, one encode launch per client {t_r1:8.1f} us")

# f1 batched: the delta of 10 clients' local models (cnn-sized tensors, 401,306 parameters) against one global model
shapes = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (2048, 123), (123,), (62, 2048), (62,)]
glob = [torch.randn(*s, generator=g, device="cuda") for s in shapes]
locs = [[t + torch.randn(*t.shape, generator=g, device="cuda") * 1e-3 for t in glob] for _ in range(10)]
n = sum(t.numel() for t in glob)
k = n // 100
t_b = tm(lambda: codec.stacked_encode_delta_batch(locs, glob, k, 127, seeds=list(range(10)), counter=1))
t_1 = tm(lambda: [codec.stacked_encode_delta(lp, glob, k, 127, seed=c, counter=1) for c, lp in enumerate(locs)])
print(f"delta-fused, 10 clients x {n:,d}: batched {t_b:8.1f} us   one launch per client {t_1:8.1f} us   "
      f"x{t_1 / t_b:.2f}")
