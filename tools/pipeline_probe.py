"""The 1 GiB headline step with the next step's encode overlapping the previous step's decode (two streams: encodes
on A, decodes on B after their encode's event; two packets alternate, a packet is re-encoded only after its decode
has run), against the one-stream step.  The last decoded vector is compared bit for bit with the one-stream run."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import codec

n = 268_435_456
k = n // 100
dev = torch.device("cuda", 0)
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1234)) * 1e-3
out = torch.empty_like(x)
pk = [codec.stacked_encode(x, k, 127, 1, 0), codec.stacked_encode(x, k, 127, 1, 0)]
sA = torch.cuda.current_stream(dev)
sB = torch.cuda.Stream(dev)
K = int(os.environ.get("STEPS", "20"))


def one_stream(c0):
    for i in range(K):
        codec.stacked_encode(x, k, 127, 1, c0 + i, out=pk[i & 1])
        codec.stacked_decode(pk[i & 1], out=out)


def two_streams(c0):
    ev_enc = [torch.cuda.Event() for _ in range(K)]
    ev_dec = [torch.cuda.Event() for _ in range(K)]
    for i in range(K):
        if i >= 2:
            sA.wait_event(ev_dec[i - 2])  # packet i & 1 was read by decode i - 2
        codec.stacked_encode(x, k, 127, 1, c0 + i, out=pk[i & 1])
        ev_enc[i].record(sA)
        with torch.cuda.stream(sB):
            sB.wait_event(ev_enc[i])
            codec.stacked_decode(pk[i & 1], out=out)
            ev_dec[i].record(sB)
    sA.wait_stream(sB)


def timed(fn, c0):
    fn(c0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(sA)
    fn(c0)
    b.record(sA)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / K


for rnd in range(3):
    for name, fn in (("one stream", one_stream), ("two streams", two_streams)):
        ms = timed(fn, 1000 * rnd)
        print(f"round {rnd} {name:12s}: {ms:.4f} ms/step  {(8 * n + 10 * k) / ms / 1e6:.0f} GB/s", flush=True)
one_stream(77)
torch.cuda.synchronize()
ref = out.view(torch.int32).clone()
out.zero_()
two_streams(77)
torch.cuda.synchronize()
print("last decoded vector bit-identical:", torch.equal(ref, out.view(torch.int32)), flush=True)
print("encoder status:", codec.topk_status_all() if hasattr(codec, "topk_status_all") else "n/a", flush=True)
