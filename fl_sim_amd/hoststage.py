"""Server state in host memory: the reference's own placement (``Server.__init__`` sets ``self.device =
torch.device("cpu")``, nodes.py:606; ``FedOptServer.update`` moves every client tensor there, _fedopt.py:205-208).

The aggregation kernels run on a HIP device, so a host-resident server's tensors are staged: copied to the device,
folded there in the same launches as a device-resident server (the same fmaf chains, so the result is bit-identical),
and copied back into the host tensors IN PLACE before the call returns.

Two ways to stage a group of host tensors (one model's parameters, the FedOpt δ or v list, SCAFFOLD's control
variates, ...):

* **Adopted** (:func:`adopt`, called by the ``Server`` mixins, which hold the server's own tensor objects): the
  tensors' storage is moved once into one pinned host buffer (``t.data = view``; same values, shapes, dtype and
  device), with a device buffer of the same layout.  Staging is then ONE host→device copy of each group's contiguous
  range and ONE device→host copy back, with no host-side packing: the reference's code keeps reading and writing the
  same tensors on the CPU, which now live in that buffer.  A group is recognised on every call by its tensors' data
  pointers (never by version counters: ``p.data.add_`` does not bump them), so any later ``t.data = ...``
  reassignment just sends that group through the packed form below and the next mixin call adopts it again.
* **Packed** (any other host tensors, e.g. the functional forms called on ``[p.data for p in ...]``): each tensor is
  copied into a cached pinned staging buffer, the buffer goes over in one copy, and the written tensors are copied
  back from it afterwards.

Messages left in host memory are packed the same way (one copy); messages on another HIP device are moved to the
fold's device.  Everything is ordered on the fold device's current stream, and the call synchronises that stream
once at the end (the caller reads the host tensors next).  There is no CPU compute path: without a HIP device this
raises.
"""

from __future__ import annotations

import collections
import contextlib
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_ALIGN = 64  # elements: every staged tensor starts 256-B aligned (fp32) in both buffers
_MAX_MIRRORS = 32


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def is_host(ts: Sequence[torch.Tensor]) -> bool:
    """True when a non-empty tensor list lives in host memory (the reference server's placement), judged by its first
    tensor (a model on one device; the staging copies any other tensor it meets)."""
    return len(ts) > 0 and isinstance(ts[0], torch.Tensor) and ts[0].is_cpu


def _layout(groups: Sequence[Sequence[torch.Tensor]]) -> Tuple[List[List[int]], List[Tuple[int, int]], int]:
    offs, ranges, total = [], [], 0
    for g in groups:
        start, o = total, []
        for t in g:
            o.append(total)
            total += _round_up(max(t.numel(), 1), _ALIGN)
        offs.append(o)
        ranges.append((start, total))
    return offs, ranges, total


def _device_for(msgs: Sequence[Sequence[torch.Tensor]]) -> torch.device:
    for m in msgs:
        for t in m:
            if isinstance(t, torch.Tensor) and t.device.type == "cuda":
                return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("fl_sim_amd aggregation needs a HIP device (there is no CPU compute path)")
    return torch.device("cuda", torch.cuda.current_device())


def _zero_copy_alias(host: torch.Tensor, device: torch.device) -> Optional[torch.Tensor]:
    """A device tensor over the pinned buffer's own memory (``_flcfold.alias``: checked to be mapped at its host
    address), or None when zero-copy staging is off (``FLC_HOST_ZEROCOPY=0``) or not available."""
    if os.environ.get("FLC_HOST_ZEROCOPY", "1") == "0":
        return None
    global ZERO_COPY_ERROR
    try:
        from . import _flcfold as mod
    except ImportError as e:
        ZERO_COPY_ERROR = f"ImportError: {e}"
        return None
    try:
        return mod.alias(host, device.index if device.index is not None else torch.cuda.current_device())
    except (RuntimeError, TypeError) as e:
        ZERO_COPY_ERROR = f"{type(e).__name__}: {e}"
        return None


class _Mirror:
    """Adopted groups: one pinned host buffer (the tensors' storage), and either a device alias of that buffer
    (zero-copy: the kernels read and write it in place over PCIe) or a device buffer of the same layout."""

    def __init__(self, groups: Sequence[Sequence[torch.Tensor]], device: torch.device):
        self.dtype = groups[0][0].dtype
        self.device = device
        self.offs, self.ranges, total = _layout(groups)
        self.host = torch.empty(max(total, 1), dtype=self.dtype, pin_memory=True)
        alias = _zero_copy_alias(self.host, device)
        self.zero_copy = alias is not None
        self.dev = alias if alias is not None else torch.empty(max(total, 1), dtype=self.dtype, device=device)
        self.shapes = [[tuple(t.shape) for t in g] for g in groups]
        for g, o in zip(groups, self.offs):
            for t, off in zip(g, o):
                view = self.host[off:off + t.numel()].view(t.shape)
                view.copy_(t.detach())
                t.data = view  # same values, shape, dtype and device: the storage is now the pinned buffer
        self.key = _ptr_key(groups)
        # the device views, made once (a view costs ~1-2 us of host time, a model has ~10-100 tensors)
        self.views = [[self.dev[off:off + _numel(s_)].view(s_) for off, s_ in zip(self.offs[gi], self.shapes[gi])]
                      for gi in range(len(groups))]
        # the read and written ranges of consecutive groups merge into one copy each way
        self.span = (self.ranges[0][0], self.ranges[-1][1])

    def dev_views(self, gi: int) -> List[torch.Tensor]:
        return self.views[gi]


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


def _ptr_key(groups: Sequence[Sequence[torch.Tensor]]) -> tuple:
    """(data pointer, element count) of every tensor: a tensor whose storage was reassigned or re-viewed to another
    size no longer matches (a view of the same size and pointer keeps its values where the mirror expects them)."""
    return tuple((t.data_ptr(), t.numel()) for g in groups for t in g)


ZERO_COPY_ERROR: Optional[str] = None  # why the last alias attempt failed (diagnostics)
_MIRRORS: "collections.OrderedDict[tuple, _Mirror]" = collections.OrderedDict()
_STAGING: Dict[Tuple[torch.dtype, int], torch.Tensor] = {}  # (dtype, slot) -> pinned staging buffer


def _lookup(groups: Sequence[Sequence[torch.Tensor]]) -> Optional[_Mirror]:
    m = _MIRRORS.get(_ptr_key(groups))
    if m is not None:
        _MIRRORS.move_to_end(m.key)
    return m


def adopt(groups: Sequence[Sequence[torch.Tensor]], device: Optional[torch.device] = None) -> Optional[_Mirror]:
    """Move the storage of a server's host-resident tensor groups into one pinned buffer with a device mirror (see the
    module docstring); a no-op returning the existing mirror when they already live there.  The groups must be host
    tensors of one floating dtype; anything else returns None (those calls then stage by packing).  Only callers that
    own the tensor objects (the ``Server`` mixins) adopt: re-pointing a temporary ``p.data`` object would leave the
    parameter itself behind."""
    groups = [list(g) for g in groups if len(g)]
    if not groups or not all(isinstance(t, torch.Tensor) and t.is_cpu for g in groups for t in g):
        return None
    dtype = groups[0][0].dtype
    if dtype not in (torch.float32, torch.float64) or any(t.dtype != dtype for g in groups for t in g):
        return None
    if len({id(t) for g in groups for t in g}) != sum(len(g) for g in groups):
        return None  # one tensor object twice: it cannot live at two offsets
    m = _lookup(groups)
    if m is not None:
        return m
    if device is None:
        device = _device_for([])
    m = _Mirror(groups, device)
    _MIRRORS[m.key] = m
    while len(_MIRRORS) > _MAX_MIRRORS:
        _MIRRORS.popitem(last=False)
    return m


def _staging(dtype: torch.dtype, slot: int, n: int) -> torch.Tensor:
    buf = _STAGING.get((dtype, slot))
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 1024), dtype=dtype, pin_memory=True)
        _STAGING[(dtype, slot)] = buf
    return buf


def stage_messages(msgs: Sequence[Sequence[torch.Tensor]], device: torch.device,
                   dtype: torch.dtype) -> Sequence[Sequence[torch.Tensor]]:
    """Every message's tensors on ``device``: device tensors there already are used as they are, host tensors are
    packed into one pinned buffer and sent in one copy, tensors on another HIP device are moved.  Stream-ordered on
    ``device``'s current stream.  Messages already on HIP devices (the reference's clients on cuda:i mod N) are
    returned as they are: the fold takes them in place or moves the ones on another device itself."""
    if all(len(m) == 0 or m[0].is_cuda for m in msgs):
        return msgs
    host = [(i, j, t) for i, m in enumerate(msgs) for j, t in enumerate(m) if t.device.type == "cpu"]
    out = [[t.detach() if (t.device == device) else None for t in m] for m in msgs]
    for i, m in enumerate(msgs):
        for j, t in enumerate(m):
            if t.device.type == "cuda" and t.device != device:
                out[i][j] = t.detach().to(device)
    if host:
        offs, total = [], 0
        for _, _, t in host:
            offs.append(total)
            total += _round_up(max(t.numel(), 1), _ALIGN)
        hb = _staging(dtype, 1, total)
        for (_, _, t), off in zip(host, offs):
            hb[off:off + t.numel()].view(t.shape).copy_(t.detach())
        db = torch.empty(total, dtype=dtype, device=device)
        db.copy_(hb[:total], non_blocking=True)
        for (i, j, t), off in zip(host, offs):
            out[i][j] = db[off:off + t.numel()].view(t.shape)
    return out


@contextlib.contextmanager
def staged(groups: Sequence[Sequence[torch.Tensor]], read: Sequence[bool], write: Sequence[bool],
           msgs: Sequence[Sequence[torch.Tensor]] = ()):
    """Stage host-resident groups for one aggregation call.  Yields ``(device groups, device messages)``; on a clean
    exit the groups marked ``write`` are copied back into the host tensors in place (and the stream synchronised).
    On an error the stream is synchronised as well; with the copy staging the host tensors are left untouched, with
    zero-copy staging the kernels that ran before the error have already updated them in place (no rollback).
    ``read[g]`` False skips the host→device copy of a group the call only writes."""
    groups = [list(g) for g in groups]
    dtype = next(t.dtype for g in groups for t in g)
    m = _lookup([g for g in groups if g])
    if m is not None and all(len(g) for g in groups):
        device = m.device
    else:
        m = None
        device = _device_for(msgs)
    with torch.cuda.device(device):
        stream = torch.cuda.current_stream(device)
        if m is not None and m.zero_copy:  # adopted, zero-copy: the kernels work on the host buffer itself
            dmsgs = stage_messages(msgs, device, dtype)
            try:  # (on an error the launches already made have written the host tensors: not rolled back)
                yield [m.dev_views(gi) for gi in range(len(groups))], dmsgs
            finally:
                stream.synchronize()
            return
        if m is not None:  # adopted: one copy of the groups' contiguous span, nothing packed on the host
            if all(read):
                a, b = m.span
                m.dev[a:b].copy_(m.host[a:b], non_blocking=True)
            else:
                for gi, rd in enumerate(read):
                    if rd:
                        a, b = m.ranges[gi]
                        m.dev[a:b].copy_(m.host[a:b], non_blocking=True)
            dgroups = [m.dev_views(gi) for gi in range(len(groups))]
            hbuf, dbuf, ranges, offs = m.host, m.dev, m.ranges, m.offs
        else:  # packed through the staging buffer
            offs, ranges, total = _layout(groups)
            hbuf = _staging(dtype, 0, total)
            dbuf = torch.empty(max(total, 1), dtype=dtype, device=device)
            for gi, g in enumerate(groups):
                if read[gi]:
                    for t, off in zip(g, offs[gi]):
                        hbuf[off:off + t.numel()].view(t.shape).copy_(t.detach())
                    a, b = ranges[gi]
                    dbuf[a:b].copy_(hbuf[a:b], non_blocking=True)
            dgroups = [[dbuf[off:off + t.numel()].view(t.shape) for t, off in zip(g, offs[gi])]
                       for gi, g in enumerate(groups)]
        dmsgs = stage_messages(msgs, device, dtype)
        try:
            yield dgroups, dmsgs
        except BaseException:
            # the host tensors stay as they were (nothing is copied back), but the H2D copies queued above may still
            # be reading the shared pinned staging buffers that the next call overwrites from the host: drain first
            stream.synchronize()
            raise
        if m is not None and all(write):
            a, b = m.span
            hbuf[a:b].copy_(dbuf[a:b], non_blocking=True)
        else:
            for gi, wr in enumerate(write):
                if wr:
                    a, b = ranges[gi]
                    hbuf[a:b].copy_(dbuf[a:b], non_blocking=True)
        stream.synchronize()
        if m is None:
            for gi, g in enumerate(groups):
                if write[gi]:
                    for t, off in zip(g, offs[gi]):
                        t.detach().copy_(hbuf[off:off + t.numel()].view(t.shape))
