"""The headline's dense decode alone (flc_stacked_decode_tiled, 1 GiB, k = 1 %): HIP-event time per call over 20
calls, and a bit-for-bit check of the output against the first call's.  Run once per decode form
(FLC_DECODE_PIPE=0: one wave per tile pair; default: the persistent pipelined waves, sparse.hip)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 28
k = n // 100
x = torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(1234), device="cuda") * 1e-3
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=1)
out = torch.empty(n, device="cuda")
codec.stacked_decode(pkt, out=out)
torch.cuda.synchronize()
ref = codec.stacked_decode(pkt)  # (a second buffer: same bits expected)
torch.cuda.synchronize()
same = torch.equal(out.view(torch.int32), ref.view(torch.int32))
h = hashlib.sha256(out.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    e0.record()
    for _ in range(20):
        codec.stacked_decode(pkt, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"decode pipe={os.environ.get('FLC_DECODE_PIPE', '1')} n={n}: {us:.1f} us/call, "
          f"{(4 * n + 5 * k + 4 * (n // 1024 + 1)) / us / 1e3:.0f} GB/s", flush=True)
print("repeatable:", same, "sha:", h)
