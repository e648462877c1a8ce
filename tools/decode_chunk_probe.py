"""The headline decode (stacked_decode over tile pointers, two 1024-output tiles per wave) with the XCD-chunked
workgroup order of sparse.hip (FLC_DECODE_CHUNK = workgroups per XCD chunk; 0 = plain order): decode alone and the
whole headline step, interleaved rounds, output checked equal to the plain order's."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

n = 1 << 28
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1234)) * 1e-3
out = torch.empty_like(x)
os.environ["FLC_DECODE_CHUNK"] = "0"
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
ref = codec.stacked_decode(pkt).clone()
ctr = [0]


def tm(fn, reps=20):
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


def step():
    ctr[0] += 1
    p = codec.stacked_encode(x, k, 127, seed=1, counter=ctr[0])
    codec.stacked_decode(p, out=out)


chunks = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,4,8,32,128").split(",")]
for _ in range(100):
    step()
res = {c: ([], []) for c in chunks}
for rnd in range(3):
    for c in chunks:
        os.environ["FLC_DECODE_CHUNK"] = str(c)
        res[c][0].append(tm(lambda: codec.stacked_decode(pkt, out=out)))
        assert torch.equal(out, ref), c
        res[c][1].append(tm(step))
for c, (d, s) in res.items():
    print(f"chunk {c:4d}: decode us " + " ".join(f"{v:6.1f}" for v in d) + "   step us " +
          " ".join(f"{v:6.1f}" for v in s), flush=True)
