"""Host-resident clients: pinned host deltas through the device codec with copy/compute overlap.

SURVEY.md §8(f) row f3.  In the reference every client's model lives on the CPU simulator, so a round moves each
client's flat delta host -> device, runs ``Compressor.compressVector`` (encode + decode, compressors.py:267-410) and
brings the decoded vector back (nodes.py:300-302 / fedopt.py:295-308 form the delta on the host).  Done one client
after another, the two PCIe copies serialise with each other and with the codec.  ``HostCodecPipeline`` keeps two
device buffer pairs and three streams:

    h2d stream:      copy client i+1 in     (needs: buffer pair (i+1) % 2 released by client i-1's compute)
    compute stream:  encode + decode client i (needs: its copy-in done, and its output buffer drained)
    d2h stream:      copy client i-1 out    (needs: client i-1's compute done)

so the host->device and device->host copies of neighbouring clients run at once (PCIe is full duplex) and the codec
hides under them.  All ordering is stream-side (events); the host only blocks in ``synchronize``.  Results are those
of the sequential path (same kernels, same seeds / counters).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import codec


class HostCodecPipeline:
    """Stacked top-k -> dithering round trip for host-resident client deltas (all of length ``n``).

    ``run(host_xs, host_outs, k, levels, seeds, counters)``: ``host_xs[i]`` (pinned fp32, length n) is encoded and
    decoded on the device; the dense decoded vector lands in ``host_outs[i]`` (pinned fp32).  Returns the device
    packets' wire sizes (bytes) per client.  Call ``synchronize()`` (or any device sync) before reading the outputs.
    """

    def __init__(self, n: int, device: Optional[torch.device] = None):
        self.n = int(n)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.x = [torch.empty(self.n, dtype=torch.float32, device=self.device) for _ in range(2)]
        self.out = [torch.empty(self.n, dtype=torch.float32, device=self.device) for _ in range(2)]
        self.s_h2d = torch.cuda.Stream(self.device)
        self.s_comp = torch.cuda.Stream(self.device)
        self.s_d2h = torch.cuda.Stream(self.device)
        self.in_free = [None, None]    # compute done with x[b]
        self.out_free = [None, None]   # d2h done with out[b]
        self._last = None

    @staticmethod
    def _check_host(t: torch.Tensor, n: int, name: str):
        if t.device.type != "cpu" or t.dtype != torch.float32 or t.numel() != n or not t.is_contiguous():
            raise ValueError(f"{name}: need a contiguous fp32 host tensor of {n} elements")
        if not t.is_pinned():
            raise ValueError(f"{name}: host tensor must be pinned (torch.empty(..., pin_memory=True))")

    def run(self, host_xs: Sequence[torch.Tensor], host_outs: Sequence[torch.Tensor], k: int, levels: int = 127,
            seeds: Optional[Sequence[int]] = None, counters: Optional[Sequence[int]] = None) -> List[int]:
        if len(host_xs) != len(host_outs):
            raise ValueError("one output per client delta")
        m = len(host_xs)
        seeds = list(seeds) if seeds is not None else [0] * m
        counters = list(counters) if counters is not None else list(range(m))
        for i in range(m):
            self._check_host(host_xs[i], self.n, f"host_xs[{i}]")
            self._check_host(host_outs[i], self.n, f"host_outs[{i}]")
        # the caller's pending work on the default stream comes first
        cur = torch.cuda.current_stream(self.device)
        for s in (self.s_h2d, self.s_comp, self.s_d2h):
            s.wait_stream(cur)
        sizes = []
        for i in range(m):
            b = i % 2
            with torch.cuda.stream(self.s_h2d):
                if self.in_free[b] is not None:
                    self.s_h2d.wait_event(self.in_free[b])
                self.x[b].copy_(host_xs[i], non_blocking=True)
                loaded = torch.cuda.Event()
                loaded.record(self.s_h2d)
            with torch.cuda.stream(self.s_comp):
                self.s_comp.wait_event(loaded)
                if self.out_free[b] is not None:
                    self.s_comp.wait_event(self.out_free[b])
                pkt = codec.stacked_encode(self.x[b], k, levels, seed=seeds[i], counter=counters[i])
                codec.stacked_decode(pkt, out=self.out[b])
                done = torch.cuda.Event()
                done.record(self.s_comp)
                self.in_free[b] = done
                sizes.append(pkt.nbytes)
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(done)
                host_outs[i].copy_(self.out[b], non_blocking=True)
                drained = torch.cuda.Event()
                drained.record(self.s_d2h)
                self.out_free[b] = drained
                self._last = drained
        return sizes

    def synchronize(self):
        if self._last is not None:
            self._last.synchronize()
