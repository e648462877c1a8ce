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
    """One client's stacked-codec wire in pinned host memory, as ONE packed record (flc_stacked_wire_layout):
    the fp32 norm, ascending int32 indices, 8-bit (sign | level) codes and the CSR tile pointers of the indices
    (the decoder's index) at fixed offsets, so that it crosses PCIe in one copy.  ``idx`` / ``codes`` / ``norm`` /
    ``tiles`` are views of the record.  ``nbytes`` is the payload (compressors.py:406-408 count the same as
    ``really_need_to_send_components``); ``record.numel()`` adds the alignment padding."""

    def __init__(self, n: int, k: int, levels: int):
        self.n, self.k, self.levels = int(n), int(k), int(levels)
        stride, off = codec.stacked_wire_layout(self.n, self.k)
        self.record = torch.empty(stride, dtype=torch.uint8, pin_memory=True)
        nt = (self.n + codec.TILE - 1) // codec.TILE + 1
        r = self.record
        self.norm = r[off["norm"]:off["norm"] + 4].view(torch.float32)
        self.idx = r[off["idx"]:off["idx"] + 4 * self.k].view(torch.int32)
        self.codes = r[off["codes"]:off["codes"] + max(self.k, 16)]
        self.tiles = r[off["tiles"]:off["tiles"] + 4 * nt].view(torch.int32)

    @property
    def nbytes(self) -> int:
        return 5 * self.k + 4 + 4 * self.tiles.numel()


class HostWirePipeline:
    """The client -> server path with only the packed wire on the return link.

    Client side (``encode``): pinned dense delta -> H2D -> stacked encode straight into a device wire record -> ONE D2H
    copy of the record (~14.5 MB per 1 GiB client at k = 1 %), instead of the dense decoded vector.  Server side
    (``decode_accumulate``): one H2D copy per client's record into a device record buffer, then ONE pass over the
    accumulator folding every client with its weight in message order (flc_stacked_fold_wires:
    ``acc = fmaf(w_i, decode_i, acc)``).  Client copies and kernels overlap on three streams; ordering is by events only.
    The accumulated result equals the device-resident fold of the same clients bit for bit (same kernels, seeds,
    counters and order).
    """

    def __init__(self, n: int, k: int, levels: int = 127, device: Optional[torch.device] = None):
        self.n, self.k, self.levels = int(n), int(k), int(levels)
        self.device = _device(device)
        self.stride = codec.stacked_wire_layout(self.n, self.k)[0]
        self.x = [torch.empty(self.n, dtype=torch.float32, device=self.device) for _ in range(2)]
        self.rec = [torch.empty(self.stride, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.s_h2d = torch.cuda.Stream(self.device)
        self.s_comp = torch.cuda.Stream(self.device)
        self.s_d2h = torch.cuda.Stream(self.device)
        self.in_free = [None, None]
        self.wire_free = [None, None]
        self._last = None
        self.srv = None  # server side: the device record buffer, grown on demand

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
                    self.s_comp.wait_event(self.wire_free[b])  # record b drained to the host
                codec.stacked_encode(self.x[b], self.k, self.levels, seed=seeds[i], counter=counters[i],
                                     wire=self.rec[b])
                done = torch.cuda.Event()
                done.record(self.s_comp)
                self.in_free[b] = done
            with torch.cuda.stream(self.s_d2h):
                self.s_d2h.wait_event(done)
                wires[i].record.copy_(self.rec[b], non_blocking=True)
                drained = torch.cuda.Event()
                drained.record(self.s_d2h)
                self.wire_free[b] = drained
                self._last = drained

    def decode_accumulate(self, wires: Sequence[HostWire], weights: Sequence[float], acc: torch.Tensor,
                          zero: bool = True) -> torch.Tensor:
        """Server side: ``acc = (0 if zero else acc)``, then ``acc = fmaf(weights[i], decode(wires[i]), acc)`` in
        order.  ``acc`` is a device fp32 tensor of n elements.  Asynchronous on the pipeline's compute stream."""
        if len(weights) != len(wires) or not wires:
            raise ValueError("one weight per wire, at least one")
        if acc.device != self.device or acc.dtype != torch.float32 or acc.numel() != self.n or not acc.is_contiguous():
            raise ValueError(f"acc must be a contiguous fp32 tensor of {self.n} elements on {self.device}")
        for i, w in enumerate(wires):
            if (w.n, w.k) != (self.n, self.k):
                raise ValueError(f"wires[{i}] has the wrong shape")
        m = len(wires)
        self._start()
        self.s_h2d.wait_stream(self.s_d2h)  # wires this pipeline produced have reached the host
        if self.srv is None or self.srv.shape[0] < m:
            self.srv = torch.empty(m, self.stride, dtype=torch.uint8, device=self.device)
        srv = self.srv
        srv.record_stream(self.s_h2d)  # (written on s_h2d, read by the fold on s_comp: both uses recorded, so a
        srv.record_stream(self.s_comp)  #  regrown buffer is not handed out while either still touches it)
        with torch.cuda.stream(self.s_h2d):
            self.s_h2d.wait_stream(self.s_comp)  # the previous fold has read the record buffer
            for i, w in enumerate(wires):
                srv[i].copy_(w.record, non_blocking=True)
            loaded = torch.cuda.Event()
            loaded.record(self.s_h2d)
        acc.record_stream(self.s_comp)
        with torch.cuda.stream(self.s_comp):
            self.s_comp.wait_event(loaded)
            codec.stacked_fold_wires(srv, list(range(m)), [float(v) for v in weights], self.n, self.k, self.levels,
                                     out=acc, accumulate=not zero)
            done = torch.cuda.Event()
            done.record(self.s_comp)
            self._last = done
        return acc

    def synchronize(self):
        if self._last is not None:
            self._last.synchronize()

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Make ``stream`` (default: the current one) wait for everything queued so far (no host block)."""
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.s_comp)
        (stream or torch.cuda.current_stream(self.device)).wait_stream(self.s_d2h)
