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


def _device(device) -> torch.device:
    d = torch.device(device) if device is not None else torch.device("cuda")
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


class HostCodecPipeline:
    """Stacked top-k -> dithering round trip for host-resident client deltas (all of length ``n``).

    ``run(host_xs, host_outs, k, levels, seeds, counters)``: ``host_xs[i]`` (pinned fp32, length n) is encoded and
    decoded on the device; the dense decoded vector lands in ``host_outs[i]`` (pinned fp32).  Returns the device
    packets' wire sizes (bytes) per client.  Call ``synchronize()`` (or any device sync) before reading the outputs.
    """

    def __init__(self, n: int, device: Optional[torch.device] = None):
        self.n = int(n)
        self.device = _device(device)
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


# ------------------------------------------------------------------------------------------- packed wire (f3)
class HostWire:
    """One client's stacked-codec wire in pinned host memory: ascending int32 indices, 8-bit (sign | level) codes,
    the fp32 norm and the CSR tile pointers of the indices (the decoder's index).  ``nbytes`` is what crosses PCIe
    (compressors.py:406-408 count the same payload as ``really_need_to_send_components``)."""

    def __init__(self, n: int, k: int, levels: int):
        self.n, self.k, self.levels = int(n), int(k), int(levels)
        self.idx = torch.empty(self.k, dtype=torch.int32, pin_memory=True)
        self.codes = torch.empty(max(self.k, 16), dtype=torch.uint8, pin_memory=True)
        self.norm = torch.empty(1, dtype=torch.float32, pin_memory=True)
        self.tiles = torch.empty((self.n + codec.TILE - 1) // codec.TILE + 1, dtype=torch.int32, pin_memory=True)

    @property
    def nbytes(self) -> int:
        return 5 * self.k + 4 + 4 * self.tiles.numel()


class HostWirePipeline:
    """The client -> server path with only the packed wire on the return link.

    Client side (``encode``): pinned dense delta -> H2D -> stacked encode -> D2H of the WIRE only (~5 bytes per kept
    entry + tile pointers: 14.5 MB per 1 GiB client at k = 1 %), instead of the dense decoded vector.  Server side
    (``decode_accumulate``): H2D of each client's wire -> stacked decode with the client's weight fused
    (``acc = fmaf(w_i, decode_i, acc)``, message order) into one device accumulator.  Copies and kernels of
    neighbouring clients overlap on three streams; ordering is by events only.  The accumulated result equals the
    device-resident fold of the same clients bit for bit (same kernels, seeds, counters and order).
    """

    def __init__(self, n: int, k: int, levels: int = 127, device: Optional[torch.device] = None):
        self.n, self.k, self.levels = int(n), int(k), int(levels)
        self.device = _device(device)
        self.x = [torch.empty(self.n, dtype=torch.float32, device=self.device) for _ in range(2)]
        self.pk = [None, None]
        self.s_h2d = torch.cuda.Stream(self.device)
        self.s_comp = torch.cuda.Stream(self.device)
        self.s_d2h = torch.cuda.Stream(self.device)
        self.in_free = [None, None]
        self.wire_free = [None, None]
        self._last = None
        # server side: two device wire buffers
        self.dw = [self._device_wire() for _ in range(2)]
        self.dw_free = [None, None]

    def _device_wire(self):
        d = self.device
        return (torch.empty(self.k, dtype=torch.int32, device=d), torch.empty(max(self.k, 16), dtype=torch.uint8, device=d),
                torch.empty(1, dtype=torch.float32, device=d),
                torch.empty((self.n + codec.TILE - 1) // codec.TILE + 1, dtype=torch.int32, device=d))

    def new_wires(self, m: int) -> List[HostWire]:
        return [HostWire(self.n, self.k, self.levels) for _ in range(m)]

    def _start(self):
        cur = torch.cuda.current_stream(self.device)
        for s in (self.s_h2d, self.s_comp, self.s_d2h):
            s.wait_stream(cur)

    def encode(self, host_xs: Sequence[torch.Tensor], wires: Sequence[HostWire], seeds: Optional[Sequence[int]] = None,
               counters: Optional[Sequence[int]] = None) -> None:
        """Client side: ``host_xs[i]`` (pinned fp32) -> ``wires[i]`` (pinned).  Asynchronous; ``synchronize()``
        before reading the wires on the host."""
        m = len(host_xs)
        if len(wires) != m:
            raise ValueError("one wire per client delta")
        seeds = list(seeds) if seeds is not None else [0] * m
        counters = list(counters) if counters is not None else list(range(m))
        for i in range(m):
            HostCodecPipeline._check_host(host_xs[i], self.n, f"host_xs[{i}]")
            if (wires[i].n, wires[i].k) != (self.n, self.k):
                raise ValueError(f"wires[{i}] has the wrong shape")
        self._start()
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
                if self.wire_free[b] is not None:
                    self.s_comp.wait_event(self.wire_free[b])  # the packet buffers of b drained to the host
                pkt = codec.stacked_encode(self.x[b], self.k, self.levels, seed=seeds[i], counter=counters[i])
                self.pk[b] = pkt
                done = torch.cuda.Event()
                done.record(self.s_comp)
                self.in_free[b] = done
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(done)
                w = wires[i]
                w.idx.copy_(pkt.idx, non_blocking=True)
                w.codes.copy_(pkt.codes, non_blocking=True)
                w.norm.copy_(pkt.norm, non_blocking=True)
                w.tiles.copy_(pkt.tiles, non_blocking=True)
                drained = torch.cuda.Event()
                drained.record(self.s_d2h)
                self.wire_free[b] = drained
                self._last = drained

    def decode_accumulate(self, wires: Sequence[HostWire], weights: Sequence[float], acc: torch.Tensor,
                          zero: bool = True) -> torch.Tensor:
        """Server side: ``acc = (0 if zero else acc)``, then ``acc = fmaf(weights[i], decode(wires[i]), acc)`` in
        order.  ``acc`` is a device fp32 tensor of n elements.  Asynchronous on the pipeline's compute stream."""
        if len(weights) != len(wires):
            raise ValueError("one weight per wire")
        if acc.device != self.device or acc.dtype != torch.float32 or acc.numel() != self.n or not acc.is_contiguous():
            raise ValueError(f"acc must be a contiguous fp32 tensor of {self.n} elements on {self.device}")
        self._start()
        self.s_h2d.wait_stream(self.s_d2h)  # wires this pipeline produced have reached the host
        acc.record_stream(self.s_comp)
        if zero:
            with torch.cuda.stream(self.s_comp):
                acc.zero_()
        for i, (w, wt) in enumerate(zip(wires, weights)):
            b = i % 2
            dw = self.dw[b]
            with torch.cuda.stream(self.s_h2d):
                if self.dw_free[b] is not None:
                    self.s_h2d.wait_event(self.dw_free[b])
                for dst, src in zip(dw, (w.idx, w.codes, w.norm, w.tiles)):
                    dst.copy_(src, non_blocking=True)
                loaded = torch.cuda.Event()
                loaded.record(self.s_h2d)
            with torch.cuda.stream(self.s_comp):
                self.s_comp.wait_event(loaded)
                pkt = codec.StackedPacket(dw[0], dw[1], dw[2], self.n, self.levels, dw[3])
                codec.stacked_decode(pkt, out=acc, weight=float(wt), accumulate=True)
                done = torch.cuda.Event()
                done.record(self.s_comp)
                self.dw_free[b] = done
                self._last = done
        return acc

    def synchronize(self):
        if self._last is not None:
            self._last.synchronize()

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Make ``stream`` (default: the current one) wait for everything queued so far (no host block)."""
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.s_comp)
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.s_d2h)
