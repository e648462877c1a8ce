"""The round-4 fault's shape, covered on purpose.

`gpurun_out/r04b_tests.log` recorded one `hipErrorIllegalAddress` in `test_host_wire_pipeline_equals_device_fold`
(n = 3,000,017: not a multiple of the 1024-output tile or of the 64 KB block step).  Between its last
synchronisation and the fault ran: the side-stream stacked encodes into wire records (HostWirePipeline.encode), the
server's fold of the copied records (flc_stacked_fold_wires) and the 5-client batched encode + fold of
dist.aggregate_round.  The fold and the decoders trust a record's CSR tile pointers to index its entries, and
`aggregate_round` folds records from a `torch.empty` block, so a tile pointer left unwritten by an encoder would
have sent the fold reading at an index taken from whatever that memory held before.  This test therefore:

- fills every record with garbage before each encode (0xAB / 0xFF bytes, as a recycled allocation may hold) and then
  checks every tile pointer of every record against the oracle's definition (tiles[t] = first j with
  idx[j] >= t * 1024, tiles[T] = k) and the kept indices ascending and in range;
- runs the single-client wire encodes on a side stream and the batched encodes (5 and 17 clients) on the default
  stream, at tails that are not multiples of the tile or the block step;
- folds the records (pipeline, batched record block) and requires the dense result bit-identical to the per-client
  decode-accumulate chain;
- runs in a child process (a fault there fails this test instead of the session) and requires every encoder error
  word 0.  (Round 4 ran it with the paired pass on and off; that pass was removed in round 5)
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from fl_sim_amd import codec, dist as fdist
from fl_sim_amd.host import HostWirePipeline

DEV = torch.device("cuda", 0)
out = []

def h(*ts):
    m = hashlib.sha256()
    for t in ts:
        m.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return m.hexdigest()

def check(idx, tiles, n, k, what):
    i = idx.cpu().numpy().astype(np.int64)
    t = tiles.cpu().numpy().astype(np.int64)
    T = (n + 1023) // 1024
    assert i.shape == (k,) and t.shape == (T + 1,), what
    assert np.all(np.diff(i) > 0) and i[0] >= 0 and i[-1] < n, what + ": kept indices not ascending / in range"
    exp = np.searchsorted(i, np.arange(T + 1, dtype=np.int64) * 1024)
    assert np.array_equal(t, exp), what + ": tile pointers differ from their definition"

for (n, k, m, seed) in ((3_000_017, 30_000, 5, 21), (1_000_003, 10_000, 17, 5), (7_340_033, 73_400, 5, 9)):
    gen = torch.Generator(device="cpu").manual_seed(n % 1009)
    hx = [(torch.randn(n, generator=gen) * 1e-3).pin_memory() for _ in range(m)]
    w = fdist.sample_weights([100 * (i + 1) for i in range(m)])
    stride, off = codec.stacked_wire_layout(n, k)
    nt = (n + 1023) // 1024 + 1
    # 1. the client side: wire encodes on the pipeline's side stream, into garbage-filled pinned records
    pipe = HostWirePipeline(n, k, 127, DEV)
    wires = pipe.new_wires(m)
    for wr in wires:
        wr.record.fill_(0xAB)
    pipe.encode(hx, wires, seeds=[seed + i for i in range(m)], counters=[2] * m)
    pipe.synchronize()
    dx = [t.to(DEV) for t in hx]
    for i in range(m):
        check(wires[i].idx, wires[i].tiles, n, k, f"pipeline wire {i}")
        pkt = codec.stacked_encode(dx[i], k, 127, seed=seed + i, counter=2)
        assert torch.equal(wires[i].idx, pkt.idx.cpu()) and torch.equal(wires[i].codes[:k], pkt.codes[:k].cpu())
        assert torch.equal(wires[i].tiles, pkt.tiles.cpu()) and torch.equal(wires[i].norm, pkt.norm.cpu())
    # 2. the server side: records copied in, one fold pass on the pipeline's compute stream
    acc = torch.empty(n, dtype=torch.float32, device=DEV)
    pipe.decode_accumulate(wires, w, acc)
    pipe.wait()
    # 3. the batched encode into a garbage-filled record block (default stream), every record checked
    for fill in (0xFF, 0xAB):
        recs = torch.full((m, stride), fill, dtype=torch.uint8, device=DEV)
        codec.stacked_encode_batch(dx, k, 127, seeds=[seed + i for i in range(m)], counter=2, wires=recs)
        for i in range(m):
            pk = codec.wire_packet(recs[i], n, k)
            check(pk.idx, pk.tiles, n, k, f"batched record {i} (fill {fill:#x})")
            assert torch.equal(pk.idx.cpu(), wires[i].idx) and torch.equal(pk.codes[:k].cpu(), wires[i].codes[:k])
    # 4. the folds against the per-client decode-accumulate chain
    exp = torch.zeros(n, dtype=torch.float32, device=DEV)
    for i in range(m):
        pkt = codec.stacked_encode(dx[i], k, 127, seed=seed + i, counter=2)
        codec.stacked_decode(pkt, out=exp, weight=w[i], accumulate=True)
    got = fdist.aggregate_round(dx, w, list(range(m)), fdist.stacked_decode_accumulate(k, seed=seed, counter=2))
    assert torch.equal(got.view(torch.int32), exp.view(torch.int32)), "aggregate_round differs from the chain"
    assert torch.equal(acc.view(torch.int32), exp.view(torch.int32)), "pipeline fold differs from the chain"
    torch.cuda.synchronize()
    out.append(h(acc, got, *[wr.record[: off["tiles"] + 4 * nt] for wr in wires]))
print("\n".join(out))
print("err", sum(codec.topk_status_all().values()))
"""


def _run() -> list:
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln and not ln.startswith("/opt")]
    assert lines[-1] == "err 0", lines[-1]
    return lines[:-1]


def test_tail_shapes_wire_records_and_batched_folds():
    torch.cuda.synchronize()
    assert len(_run()) == 3
