"""Device-side functional API over the C ABI: torch tensors in HBM in, torch tensors out.

Every function here launches hand-written gfx950 kernels from ``libflcodec.so`` on the current HIP
stream of the tensor's device; none of them synchronises the stream.  Tensors must be fp32, on a HIP
device and contiguous (non-contiguous or misaligned inputs are copied once).  This module is the
plumbing under :class:`fl_sim_amd.compressors.Compressor` and :mod:`fl_sim_amd.aggregation`; bench.py
drives it directly for the device-resident measurement.
"""

from __future__ import annotations

import collections.abc as _abc
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import call

_WS: Dict[Tuple[int, int, str], torch.Tensor] = {}


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device: torch.device) -> int:
    """The raw handle of ``device``'s current stream (torch's C accessor when present: building a Stream object per
    call cost a few microseconds of host time on every launch of the small configs)."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _dev_f32(x: torch.Tensor, name: str = "x") -> torch.Tensor:
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
        raise TypeError(f"{name} must be a torch tensor on a HIP device (got {type(x).__name__}"
                        f"{'' if not isinstance(x, torch.Tensor) else ' on ' + str(x.device)})")
    if x.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {x.dtype}); the codec path is fp32")
    if not x.is_contiguous() or x.data_ptr() % 16 != 0:
        x = x.contiguous().clone()
    return x


TILE = 1024  # FLC_TILE (include/flcodec.h)


_WS_SIZE: Dict[tuple, int] = {}


def _ws_size(device: torch.device, name: str, *args) -> int:
    """A workspace-size entry point's result for ``device`` (the size functions read the current device's CU count,
    so the query runs with ``device`` current), memoised per device: one ctypes call fewer per encode."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, name) + args
    v = _WS_SIZE.get(key)
    if v is None:
        with torch.cuda.device(idx):
            v = _WS_SIZE[key] = _lib.size(name, *args)
    return v


def workspace(device: torch.device, nbytes: int, kind: str) -> torch.Tensor:
    """Zero-initialised workspace, cached per (device, stream, kind) and grown on demand."""
    key = (device.index if device.index is not None else torch.cuda.current_device(), _stream(device), kind)
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _WS[key] = t
    return t


def code_bits(levels: int) -> int:
    """Bits per element of the dithering wire: sign + ceil(log2(levels + 1)), rounded up to 2/4/8."""
    b = 1 + int(math.ceil(math.log2(levels + 1)))
    for c in (2, 4, 8):
        if b <= c:
            return c
    raise ValueError(f"levels={levels} does not fit an 8-bit code (at most 127 levels)")


# ----------------------------------------------------------------------------------------------- dither
@dataclass
class QuantPacket:
    """Wire of the dense dithering codec: per-row fp32 norm + packed ``bits``-bit codes."""

    codes: torch.Tensor
    norms: torch.Tensor
    rows: int
    d: int
    kind: int
    levels: int
    bits: int
    nnz: Optional[torch.Tensor] = None

    @property
    def nbytes(self) -> int:
        return self.codes.numel() + 4 * self.rows


def quant_norm(x2d: torch.Tensor, p: float = math.inf) -> torch.Tensor:
    x2d = _dev_f32(x2d)
    rows, d = x2d.shape
    pk = _lib.FLC_NORM_INF if math.isinf(p) else (_lib.FLC_NORM_L2 if p == 2 else None)
    if pk is None:
        raise ValueError(f"p must be inf or 2 (got {p})")
    norms = torch.empty(rows, dtype=torch.float32, device=x2d.device)
    nb = _ws_size(x2d.device, "flc_quant_workspace_size", rows, d)
    ws = workspace(x2d.device, nb, "quant")
    call("flc_quant_norm", _p(x2d), rows, d, pk, _p(norms), _p(ws), ws.numel(), _stream(x2d.device))
    return norms


def count_consumers(x2d: torch.Tensor, norms: Optional[torch.Tensor]) -> torch.Tensor:
    """Device int64 scalar: the number of uniforms the reference draws for this batch."""
    x2d = _dev_f32(x2d)
    rows, d = x2d.shape
    out = torch.empty(1, dtype=torch.int64, device=x2d.device)
    call("flc_count_consumers", _p(x2d), rows, d, _p(norms), _p(out), _stream(x2d.device))
    return out


def quant_encode(x2d: torch.Tensor, kind: int, levels: int, norms: torch.Tensor, seed: int = 0, counter: int = 0,
                 compat_u: Optional[torch.Tensor] = None, want_nnz: bool = True) -> QuantPacket:
    x2d = _dev_f32(x2d)
    rows, d = x2d.shape
    bits = code_bits(levels)
    nbytes = (rows * d * bits + 7) // 8
    codes = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=x2d.device)
    nnz = torch.empty(rows, dtype=torch.int64, device=x2d.device) if want_nnz else None
    if compat_u is not None and compat_u.dtype != torch.float64:
        raise TypeError("compat_u must be float64")
    nb = _ws_size(x2d.device, "flc_quant_workspace_size", rows, d)
    ws = workspace(x2d.device, nb, "quant")
    call("flc_quant_encode", _p(x2d), rows, d, kind, levels, bits, _p(norms), seed, counter, _p(compat_u),
         _p(codes), _p(nnz), _p(ws), ws.numel(), _stream(x2d.device))
    return QuantPacket(codes, norms, rows, d, kind, levels, bits, nnz)


def quant_encode_decode(x2d: torch.Tensor, kind: int, levels: int, norms: torch.Tensor, seed: int = 0,
                        counter: int = 0, compat_u: Optional[torch.Tensor] = None, want_nnz: bool = True,
                        out: Optional[torch.Tensor] = None) -> Tuple[QuantPacket, torch.Tensor]:
    """quant_encode and quant_decode in one pass (flc_quant_encode_decode): the same codes, and the decoded batch
    computed from each code as it is made.  Returns (packet, decoded [rows, d])."""
    x2d = _dev_f32(x2d)
    rows, d = x2d.shape
    bits = code_bits(levels)
    codes = torch.empty(max((rows * d * bits + 7) // 8, 1), dtype=torch.uint8, device=x2d.device)
    nnz = torch.empty(rows, dtype=torch.int64, device=x2d.device) if want_nnz else None
    if out is None:
        out = torch.empty(rows, d, dtype=torch.float32, device=x2d.device)
    if compat_u is not None and compat_u.dtype != torch.float64:
        raise TypeError("compat_u must be float64")
    ws = workspace(x2d.device, _ws_size(x2d.device, "flc_quant_workspace_size", rows, d), "quant")
    call("flc_quant_encode_decode", _p(x2d), rows, d, kind, levels, bits, _p(norms), seed, counter, _p(compat_u),
         _p(codes), _p(nnz), _p(out), _p(ws), ws.numel(), _stream(x2d.device))
    return QuantPacket(codes, norms, rows, d, kind, levels, bits, nnz), out


def quant_encode_auto(x2d: torch.Tensor, kind: int, levels: int, p: float = math.inf, seed: int = 0, counter: int = 0,
                      want_nnz: bool = False, decode: bool = True):
    """Philox mode with the norm included (flc_quant_encode_auto): norm, encode and (``decode``) the decoded batch in
    two launches for rows of >= 2048 elements.  Returns (packet, decoded or None)."""
    x2d = _dev_f32(x2d)
    rows, d = x2d.shape
    pk = _lib.FLC_NORM_INF if math.isinf(p) else (_lib.FLC_NORM_L2 if p == 2 else None)
    if pk is None:
        raise ValueError(f"p must be inf or 2 (got {p})")
    bits = code_bits(levels)
    codes = torch.empty(max((rows * d * bits + 7) // 8, 1), dtype=torch.uint8, device=x2d.device)
    norms = torch.empty(rows, dtype=torch.float32, device=x2d.device)
    nnz = torch.empty(rows, dtype=torch.int64, device=x2d.device) if want_nnz else None
    out = torch.empty(rows, d, dtype=torch.float32, device=x2d.device) if decode else None
    ws = workspace(x2d.device, _ws_size(x2d.device, "flc_quant_workspace_size", rows, d), "quant")
    call("flc_quant_encode_auto", _p(x2d), rows, d, kind, levels, bits, pk, seed, counter, _p(codes), _p(norms),
         _p(nnz), _p(out), _p(ws), ws.numel(), _stream(x2d.device))
    _after_encode(x2d.device, ("quant",))
    return QuantPacket(codes, norms, rows, d, kind, levels, bits, nnz), out


def quant_decode(pkt: QuantPacket, out: Optional[torch.Tensor] = None, row_weights: Optional[torch.Tensor] = None,
                 accumulate: bool = False) -> torch.Tensor:
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an out tensor")
        out = torch.empty(pkt.rows, pkt.d, dtype=torch.float32, device=pkt.codes.device)
    call("flc_quant_decode", _p(pkt.codes), pkt.rows, pkt.d, pkt.kind, pkt.levels, pkt.bits, _p(pkt.norms),
         _p(row_weights), int(accumulate), _p(out), _stream(out.device))
    return out


# ---------------------------------------------------------------------------------------------- natural
def natural_encode(x: torch.Tensor, seed: int = 0, counter: int = 0, compat_u: Optional[torch.Tensor] = None,
                   want_nnz: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    x = _dev_f32(x).reshape(-1)
    n = x.numel()
    codes = torch.empty(n, dtype=torch.int16, device=x.device)
    nnz = torch.empty(1, dtype=torch.int64, device=x.device) if want_nnz else None
    nb = _ws_size(x.device, "flc_natural_workspace_size", n)
    ws = workspace(x.device, nb, "natural")
    call("flc_natural_encode", _p(x), n, seed, counter, _p(compat_u), _p(codes), _p(nnz), _p(ws), ws.numel(),
         _stream(x.device))
    return codes, nnz


def natural_decode(codes: torch.Tensor, n: int, out: Optional[torch.Tensor] = None, weight: float = 1.0,
                   accumulate: bool = False) -> torch.Tensor:
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=codes.device)
    call("flc_natural_decode", _p(codes), n, weight, int(accumulate), _p(out), _stream(out.device))
    return out


# ------------------------------------------------------------------------------------------------ top-k
# FLC_TOPK_CHECK=1: read the persistent encoder's sticky error word after every top-k / stacked encode
# (one host synchronisation per call) and raise if a call lost co-residency (include/flcodec.h)
TOPK_CHECK = os.environ.get("FLC_TOPK_CHECK", "0") not in ("", "0")
TOPK_ERRORS = {1: "digit not found", 2: "count mismatch", 4: "exchange spin timeout"}
_TOPK_KINDS = ("topk", "topk_batch")  # single-client and batched encoder workspaces (never shared)
# every workspace kind whose kernels run a grid exchange, and the entry point reading its sticky error word
_STATUS_FN = {"topk": "flc_topk_status", "topk_batch": "flc_topk_status", "quant": "flc_quant_status",
              "f64": "flc_f64_status"}


def _status(device: torch.device, kinds: Sequence[str], reset: bool = True) -> int:
    err = 0
    for kind in kinds:
        key = (device.index if device.index is not None else torch.cuda.current_device(), _stream(device), kind)
        ws = _WS.get(key)
        if ws is None:
            continue
        out = torch.empty(1, dtype=torch.int64, device=device)
        call(_STATUS_FN[kind], _p(ws), _p(out), int(reset), _stream(device))
        err |= int(out.item())
    return err


def topk_status(device: Optional[torch.device] = None, reset: bool = True) -> int:
    """The sticky error word of the top-k workspace of ``device``'s current stream (0 = every encode since
    the last reset was exact).  Synchronises that stream."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    return _status(device, _TOPK_KINDS, reset)


def quant_status(device: Optional[torch.device] = None, reset: bool = True) -> int:
    """The sticky error word of the one-launch quantizer's workspace (quant_fused_kernel's grid exchange) of
    ``device``'s current stream; 0 = every call since the last reset had all its blocks resident."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    return _status(device, ("quant",), reset)


def topk_status_all(reset: bool = True) -> Dict[Tuple[int, int], int]:
    """{(device, stream): error word} of every cached workspace whose kernels run a grid exchange (the top-k
    encoders, the one-launch quantizer).  Synchronises each device first and reads on its current stream (the stream
    a workspace was used on may be gone)."""
    res: Dict[Tuple[int, int], int] = {}
    for (dev, stream, kind), ws in list(_WS.items()):
        if kind not in _STATUS_FN:
            continue
        d = torch.device("cuda", dev)
        torch.cuda.synchronize(d)
        out = torch.empty(1, dtype=torch.int64, device=d)
        call(_STATUS_FN[kind], _p(ws), _p(out), int(reset), _stream(d))
        res[(dev, stream)] = res.get((dev, stream), 0) | int(out.item())
    return res


def _after_encode(device: torch.device, kinds: Sequence[str] = _TOPK_KINDS) -> None:
    """FLC_TOPK_CHECK: read the sticky error word of the workspaces ``kinds`` (one host synchronisation) and raise
    if a grid-exchange launch lost co-residency; its output would be wrong."""
    if TOPK_CHECK:
        err = _status(device, kinds)
        if err:
            bits = ", ".join(v for b, v in TOPK_ERRORS.items() if err & b)
            what = {("quant",): "quantizer", ("f64",): "float64 top-k select"}.get(tuple(kinds), "top-k encode")
            raise _lib.FlcError(f"{what} lost co-residency or failed ({bits}); its output may be wrong")


def _tiles(n: int, device: torch.device) -> torch.Tensor:
    """CSR tile pointers over FLC_TILE-output tiles (include/flcodec.h)."""
    return torch.empty((n + TILE - 1) // TILE + 1, dtype=torch.int32, device=device)


def topk_encode(x: torch.Tensor, k: int, with_tiles: bool = False):
    """Kept set of the reference Top-K (k largest signed values): (idx int32 ascending, val fp32), plus the
    tile pointers of idx when ``with_tiles`` (emitted by the encoder, saving the decoder an index pass)."""
    x = _dev_f32(x).reshape(-1)
    n = x.numel()
    idx = torch.empty(k, dtype=torch.int32, device=x.device)
    val = torch.empty(k, dtype=torch.float32, device=x.device)
    tiles = _tiles(n, x.device) if with_tiles else None
    ws = workspace(x.device, _ws_size(x.device, "flc_topk_workspace_size", n, k), "topk")
    call("flc_topk_encode_tiled", _p(x), n, k, _p(idx), _p(val), _p(tiles), _p(ws), ws.numel(), _stream(x.device))
    _after_encode(x.device)
    return (idx, val, tiles) if with_tiles else (idx, val)


def topk_encode_batch(xs: Sequence[torch.Tensor], k: int, with_tiles: bool = False):
    """The top-k of many clients' flat deltas (one size) in one launch (flc_topk_encode_batch): entry c equals
    ``topk_encode(xs[c], k, with_tiles)``."""
    import ctypes

    xs = [_dev_f32(x).reshape(-1) for x in xs]
    C = len(xs)
    if C == 0:
        return []
    n, dev = xs[0].numel(), xs[0].device
    if any(x.numel() != n or x.device != dev for x in xs):
        raise ValueError("a batched encode takes clients of one size on one device")
    ntl = (n + TILE - 1) // TILE + 1
    idx = torch.empty(C, k, dtype=torch.int32, device=dev)
    val = torch.empty(C, k, dtype=torch.float32, device=dev)
    tiles = torch.empty(C, ntl, dtype=torch.int32, device=dev) if with_tiles else None
    P = ctypes.c_void_p * C
    vp = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    ws = workspace(dev, _ws_size(dev, "flc_topk_encode_batch_workspace_size", n, k, C), "topk_batch")
    call("flc_topk_encode_batch", vp(P(*[x.data_ptr() for x in xs])), C, n, k,
         vp(P(*[idx.data_ptr() + 4 * k * c for c in range(C)])), vp(P(*[val.data_ptr() + 4 * k * c for c in range(C)])),
         vp(P(*[tiles.data_ptr() + 4 * ntl * c for c in range(C)])) if with_tiles else None, _p(ws), ws.numel(),
         _stream(dev))
    _after_encode(dev)
    rows = zip(idx.unbind(0), val.unbind(0), tiles.unbind(0) if with_tiles else [None] * C)
    return [(i_, v_, t_) if with_tiles else (i_, v_) for i_, v_, t_ in rows]


def sparse_decode(idx: torch.Tensor, val: torch.Tensor, n: int, scale: float = 1.0, out: Optional[torch.Tensor] = None,
                  weight: float = 1.0, accumulate: bool = False, tiles: Optional[torch.Tensor] = None) -> torch.Tensor:
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=val.device)
    if tiles is not None:
        call("flc_sparse_decode_tiled", _p(idx), _p(val), idx.numel(), scale, n, weight, int(accumulate), _p(out),
             _p(tiles), _stream(out.device))
        return out
    ws = workspace(out.device, _ws_size(out.device, "flc_sparse_decode_workspace_size", n), "decode")
    call("flc_sparse_decode", _p(idx), _p(val), idx.numel(), scale, n, weight, int(accumulate), _p(out), _p(ws),
         ws.numel(), _stream(out.device))
    return out


@dataclass
class StackedPacket:
    """Wire of the stacked codec: ascending int32 indices, 8-bit (sign | level) codes, fp32 norm; plus the
    encoder-emitted tile pointers of the indices (CSR over 1024-output tiles), the decoder's index."""

    idx: torch.Tensor
    codes: torch.Tensor
    norm: torch.Tensor
    n: int
    levels: int
    tiles: Optional[torch.Tensor] = None

    @property
    def nbytes(self) -> int:
        return 5 * self.idx.numel() + 4 + (4 * self.tiles.numel() if self.tiles is not None else 0)


class PacketBatch(_abc.Sequence):
    """The packets of a batched encode (one row per client of four [clients, ...] blocks), made on demand: packet c
    is ``StackedPacket(idx[c], codes[c], norm[c], n, levels, tiles[c])``.  A round of many small clients would
    otherwise spend more host time building views than the GPU spends encoding (4 views x 100 clients)."""

    def __init__(self, idx, codes, norm, tiles, n: int, levels: int):
        self.idx, self.codes, self.norm, self.tiles, self.n, self.levels = idx, codes, norm, tiles, n, levels

    def __len__(self) -> int:
        return self.idx.shape[0]

    def __getitem__(self, c):
        if isinstance(c, slice):
            return [self[i] for i in range(*c.indices(len(self)))]
        if c < 0:
            c += len(self)
        if not 0 <= c < len(self):
            raise IndexError(c)
        return StackedPacket(self.idx[c], self.codes[c], self.norm[c], self.n, self.levels,
                             None if self.tiles is None else self.tiles[c])


def _batch_ptrs(xs: Sequence[torch.Tensor], n: int, dev: torch.device) -> Optional[List[int]]:
    """The clients' data pointers when every one is a contiguous, 16-B aligned fp32 tensor of n elements on `dev`
    (one lean pass: the batch may hold hundreds of clients); None otherwise."""
    f32, di = torch.float32, dev.index
    out = []
    for x in xs:
        if not (isinstance(x, torch.Tensor) and x.dtype is f32 and x.numel() == n and x.is_contiguous()
                and x.get_device() == di):
            return None
        p = x.data_ptr()
        if p & 15:
            return None
        out.append(p)
    return out


_WIRE_LAYOUT = {}


def stacked_wire_layout(n: int, k: int):
    """(record bytes, {"norm", "idx", "codes", "tiles"} byte offsets) of the packed stacked wire
    (flc_stacked_wire_layout): one contiguous record per client whose layout depends on (n, k) only."""
    import ctypes

    key = (int(n), int(k))
    r = _WIRE_LAYOUT.get(key)
    if r is None:
        off = (ctypes.c_int64 * 4)()
        total = _lib.size("flc_stacked_wire_layout", int(n), int(k), ctypes.cast(off, ctypes.c_void_p))
        if total == 0:
            raise ValueError(f"bad wire shape n={n}, k={k}")
        r = (int(total), dict(zip(("norm", "idx", "codes", "tiles"), (int(v) for v in off))))
        _WIRE_LAYOUT[key] = r
    return r


def wire_packet(record: torch.Tensor, n: int, k: int, levels: int = 127) -> StackedPacket:
    """The StackedPacket whose tensors are views into one packed wire record (a uint8 HIP tensor of at least
    ``stacked_wire_layout(n, k)[0]`` bytes, 16-B aligned)."""
    stride, off = stacked_wire_layout(n, k)
    if record.dtype != torch.uint8 or record.device.type != "cuda" or not record.is_contiguous():
        raise TypeError("a wire record is a contiguous uint8 HIP tensor")
    rec = record.reshape(-1)
    if rec.numel() < stride or rec.data_ptr() % 16 != 0:
        raise ValueError(f"a wire record needs {stride} bytes, 16-B aligned")
    ntiles = (n + TILE - 1) // TILE + 1
    return StackedPacket(rec[off["idx"]:off["idx"] + 4 * k].view(torch.int32),
                         rec[off["codes"]:off["codes"] + max(k, 16)],
                         rec[off["norm"]:off["norm"] + 4].view(torch.float32), int(n), int(levels),
                         rec[off["tiles"]:off["tiles"] + 4 * ntiles].view(torch.int32))


def stacked_encode(x: torch.Tensor, k: int, levels: int = 127, seed: int = 0, counter: int = 0,
                   with_tiles: bool = True, wire: Optional[torch.Tensor] = None,
                   out: Optional[StackedPacket] = None) -> StackedPacket:
    """Stacked top-k -> 8-bit dithering encode.  ``wire``: a packed wire record (see :func:`wire_packet`) to write
    the packet into; the returned packet's tensors are then views of it.  ``out``: a packet of the same (n, k) whose
    tensors are overwritten (no allocation per call); it is returned."""
    x = _dev_f32(x).reshape(-1)
    n = x.numel()
    if out is not None:
        if out.n != n or out.idx.numel() != k or out.idx.device != x.device or (with_tiles and out.tiles is None):
            raise ValueError("`out` must be a packet of the same n and k on the input's device")
        idx, codes, norm, tiles = out.idx, out.codes, out.norm, out.tiles if with_tiles else None
    elif wire is not None:
        if wire.device != x.device:
            raise ValueError("the wire record must be on the input's device")
        pk = wire_packet(wire, n, k, levels)
        idx, codes, norm, tiles = pk.idx, pk.codes, pk.norm, pk.tiles
    else:
        idx = torch.empty(k, dtype=torch.int32, device=x.device)
        codes = torch.empty(max(k, 16), dtype=torch.uint8, device=x.device)
        norm = torch.empty(1, dtype=torch.float32, device=x.device)
        tiles = _tiles(n, x.device) if with_tiles else None
    ws = workspace(x.device, _ws_size(x.device, "flc_topk_workspace_size", n, k), "topk")
    call("flc_stacked_encode_tiled", _p(x), n, k, levels, seed, counter, None, _p(idx), _p(codes), _p(norm),
         _p(tiles), _p(ws), ws.numel(), _stream(x.device))
    _after_encode(x.device)
    return StackedPacket(idx, codes, norm, n, levels, tiles)


def stacked_encode_batch(xs: Sequence[torch.Tensor], k: int, levels: int = 127, seeds: Sequence[int] = (),
                         counter: int = 0, with_tiles: bool = True, wires=None) -> Optional[Sequence[StackedPacket]]:
    """The stacked encode of many clients' flat deltas (all of one size) in one launch (flc_stacked_encode_batch):
    packet c equals ``stacked_encode(xs[c], k, levels, seeds[c], counter)`` bit for bit.  ``wires``: the packed wire
    records to write into — a ``[clients, >= stride]`` uint8 tensor (then nothing is returned: the records are the
    output) or a list of one record per client (the packets returned are views of them)."""
    import ctypes

    C = len(xs)
    if C == 0:
        return []
    x0 = xs[0]
    n, dev = x0.numel(), x0.device
    xp = _batch_ptrs(xs, n, dev) if dev.type == "cuda" else None
    if xp is None:  # (the slow path: checks with messages, copies of misaligned inputs)
        xs = [_dev_f32(x).reshape(-1) for x in xs]
        if any(x.numel() != n or x.device != dev for x in xs):
            raise ValueError("a batched encode takes clients of one size on one device")
        xp = [x.data_ptr() for x in xs]
    seeds = list(seeds) if len(seeds) else [0] * C
    if len(seeds) != C:
        raise ValueError("one seed per client")
    P = ctypes.c_void_p * C
    stride, off = stacked_wire_layout(n, k)
    pks = None
    if isinstance(wires, torch.Tensor):  # one [C, >= stride] record block: pointers by arithmetic
        if (wires.dtype != torch.uint8 or wires.dim() != 2 or wires.shape[0] != C or wires.shape[1] < stride
                or not wires.is_contiguous() or wires.device != dev or wires.data_ptr() % 16 or wires.shape[1] % 16):
            raise ValueError(f"records must be a contiguous [{C}, >= {stride}] uint8 block (16-B rows) on {dev}")
        rs = wires.shape[1]
        bases = [wires.data_ptr() + c * rs for c in range(C)]
        ptr = {f: P(*[b + off[f] for b in bases]) for f in ("idx", "codes", "norm", "tiles")}
    else:
        if wires is not None:
            if len(wires) != C:
                raise ValueError("one wire record per client")
            pks = [wire_packet(r, n, k, levels) for r in wires]
            ptr = {"idx": P(*[p.idx.data_ptr() for p in pks]), "codes": P(*[p.codes.data_ptr() for p in pks]),
                   "norm": P(*[p.norm.data_ptr() for p in pks]), "tiles": P(*[p.tiles.data_ptr() for p in pks])}
        else:  # one block per field, the packets its rows (views made in one unbind each)
            ntl = (n + TILE - 1) // TILE + 1
            kc = max(k, 16)
            idx = torch.empty(C, k, dtype=torch.int32, device=dev)
            codes = torch.empty(C, kc, dtype=torch.uint8, device=dev)
            norm = torch.empty(C, 1, dtype=torch.float32, device=dev)
            tiles = torch.empty(C, ntl, dtype=torch.int32, device=dev) if with_tiles else None
            pks = PacketBatch(idx, codes, norm, tiles, n, levels)
            b = {f: t.data_ptr() for f, t in (("idx", idx), ("codes", codes), ("norm", norm))}
            ptr = {"idx": P(*[b["idx"] + 4 * k * c for c in range(C)]),
                   "codes": P(*[b["codes"] + kc * c for c in range(C)]),
                   "norm": P(*[b["norm"] + 4 * c for c in range(C)]),
                   "tiles": P(*[tiles.data_ptr() + 4 * ntl * c for c in range(C)]) if with_tiles else None}
    ws = workspace(dev, _ws_size(dev, "flc_stacked_encode_batch_workspace_size", n, k, C), "topk_batch")
    vp = lambda a: None if a is None else ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    call("flc_stacked_encode_batch", vp(P(*xp)), C, n, k, levels,
         vp((ctypes.c_uint64 * C)(*[int(s_) for s_ in seeds])), counter, vp(ptr["idx"]), vp(ptr["codes"]),
         vp(ptr["norm"]), vp(ptr["tiles"]), _p(ws), ws.numel(), _stream(dev))
    _after_encode(dev)
    return pks


def stacked_encode_delta_batch(local_params: Sequence[Sequence[torch.Tensor]], global_params: Sequence[torch.Tensor],
                               k: int, levels: int = 127, seeds: Sequence[int] = (),
                               counter: int = 0) -> "PacketBatch":
    """The delta-fused stacked encode of a round's clients in one launch (flc_stacked_encode_delta_batch): client c's
    delta ``cat([l - g for l, g in zip(local_params[c], global_params)])`` (the global model shared by every client),
    packet c equal to ``stacked_encode_delta(local_params[c], global_params, k, levels, seeds[c], counter)``."""
    import ctypes

    C = len(local_params)
    if C == 0:
        return []
    ok = lambda t: t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 4 == 0  # noqa: E731
    gs = [t if ok(t) else t.contiguous().float() for t in global_params]
    ls = [[t if ok(t) else t.contiguous().float() for t in lp] for lp in local_params]
    m = len(gs)
    if m == 0 or any(len(lp) != m for lp in ls):
        raise ValueError("every client has one local tensor per global tensor, at least one")
    dev = gs[0].device
    for lp in ls:
        for a, b in zip(lp, gs):
            if a.numel() != b.numel() or a.device != dev or b.device != dev or dev.type != "cuda":
                raise ValueError("local and global tensors must be HIP tensors of matching sizes on one device")
    n = sum(t.numel() for t in gs)
    seeds = list(seeds) if len(seeds) else [0] * C
    if len(seeds) != C:
        raise ValueError("one seed per client")
    ntl = (n + TILE - 1) // TILE + 1
    kc = max(k, 16)
    idx = torch.empty(C, k, dtype=torch.int32, device=dev)
    codes = torch.empty(C, kc, dtype=torch.uint8, device=dev)
    norm = torch.empty(C, 1, dtype=torch.float32, device=dev)
    tiles = torch.empty(C, ntl, dtype=torch.int32, device=dev)
    P = ctypes.c_void_p
    vp = lambda a: ctypes.cast(a, P)  # noqa: E731
    ws = workspace(dev, _ws_size(dev, "flc_stacked_encode_delta_batch_workspace_size", n, k, C, m), "topk_batch")
    call("flc_stacked_encode_delta_batch", vp((P * (C * m))(*[t.data_ptr() for lp in ls for t in lp])),
         vp((P * m)(*[t.data_ptr() for t in gs])), vp((ctypes.c_int64 * m)(*[t.numel() for t in gs])), m, C, k,
         levels, vp((ctypes.c_uint64 * C)(*[int(s_) for s_ in seeds])), counter,
         vp((P * C)(*[idx.data_ptr() + 4 * k * c for c in range(C)])),
         vp((P * C)(*[codes.data_ptr() + kc * c for c in range(C)])),
         vp((P * C)(*[norm.data_ptr() + 4 * c for c in range(C)])),
         vp((P * C)(*[tiles.data_ptr() + 4 * ntl * c for c in range(C)])), _p(ws), ws.numel(), _stream(dev))
    _after_encode(dev)
    return PacketBatch(idx, codes, norm, tiles, n, levels)


def stacked_encode_delta(local_params: Sequence[torch.Tensor], global_params: Sequence[torch.Tensor], k: int,
                         levels: int = 127, seed: int = 0, counter: int = 0,
                         wire: Optional[torch.Tensor] = None) -> StackedPacket:
    """The stacked encode of the client delta ``cat([l - g for l, g in zip(local, global)])`` with the delta formed in
    the encoder's read pass (flc_stacked_encode_delta): the flat delta is never written.  Same packet as
    ``stacked_encode(delta_flatten(local, global), ...)``.  ``wire``: a packed wire record to write into (the packet's
    tensors are then views of it, see :func:`wire_packet`)."""
    import ctypes

    ls = [t if (t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 4 == 0) else t.contiguous().float()
          for t in local_params]
    gs = [t if (t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 4 == 0) else t.contiguous().float()
          for t in global_params]
    if len(ls) != len(gs) or not ls:
        raise ValueError("one global tensor per local tensor, at least one")
    for a, b in zip(ls, gs):
        if a.numel() != b.numel() or a.device != b.device or a.device.type != "cuda":
            raise ValueError("local and global tensors must be HIP tensors of matching sizes")
    dev = ls[0].device
    n = sum(t.numel() for t in ls)
    m = len(ls)
    lp = (ctypes.c_void_p * m)(*[t.data_ptr() for t in ls])
    gp = (ctypes.c_void_p * m)(*[t.data_ptr() for t in gs])
    sz = (ctypes.c_int64 * m)(*[t.numel() for t in ls])
    if wire is not None:
        if wire.device != dev:
            raise ValueError("the wire record must be on the tensors' device")
        pk = wire_packet(wire, n, k, levels)
        idx, codes, norm, tiles = pk.idx, pk.codes, pk.norm, pk.tiles
    else:
        idx = torch.empty(k, dtype=torch.int32, device=dev)
        codes = torch.empty(max(k, 16), dtype=torch.uint8, device=dev)
        norm = torch.empty(1, dtype=torch.float32, device=dev)
        tiles = _tiles(n, dev)
    ws = workspace(dev, _ws_size(dev, "flc_stacked_encode_delta_workspace_size", n, k, m), "topk")
    call("flc_stacked_encode_delta", ctypes.cast(lp, ctypes.c_void_p), ctypes.cast(gp, ctypes.c_void_p),
         ctypes.cast(sz, ctypes.c_void_p), m, k, levels, seed, counter, _p(idx), _p(codes), _p(norm), _p(tiles), _p(ws),
         ws.numel(), _stream(dev))
    _after_encode(dev)
    return StackedPacket(idx, codes, norm, n, levels, tiles)


def stacked_decode(pkt: StackedPacket, out: Optional[torch.Tensor] = None, weight: float = 1.0,
                   accumulate: bool = False) -> torch.Tensor:
    if out is None:
        out = torch.empty(pkt.n, dtype=torch.float32, device=pkt.idx.device)
    if pkt.tiles is not None:
        call("flc_stacked_decode_tiled", _p(pkt.idx), _p(pkt.codes), pkt.idx.numel(), pkt.levels, _p(pkt.norm), pkt.n,
             weight, int(accumulate), _p(out), _p(pkt.tiles), _stream(out.device))
        return out
    ws = workspace(out.device, _ws_size(out.device, "flc_sparse_decode_workspace_size", pkt.n), "decode")
    call("flc_stacked_decode", _p(pkt.idx), _p(pkt.codes), pkt.idx.numel(), pkt.levels, _p(pkt.norm), pkt.n, weight,
         int(accumulate), _p(out), _p(ws), ws.numel(), _stream(out.device))
    return out


def stacked_fold_wires(wires: torch.Tensor, slots: Sequence[int], weights: Sequence[float], n: int, k: int,
                       levels: int = 127, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """Server fold of many clients' packed wires in one pass (flc_stacked_fold_wires):
    ``out = (out if accumulate else +0)``, then ``out = fmaf(weights[c], decode(wires[slots[c]]), out)`` for c in
    order — bit-identical to zeroing ``out`` and calling ``stacked_decode(..., weight, accumulate=True)`` per client.
    ``wires``: uint8 HIP tensor [records, stride] (or flat, records of ``stacked_wire_layout(n, k)[0]`` bytes)."""
    import ctypes

    stride, _ = stacked_wire_layout(n, k)
    if wires.dtype != torch.uint8 or wires.device.type != "cuda" or not wires.is_contiguous():
        raise TypeError("wires must be a contiguous uint8 HIP tensor")
    if wires.dim() == 2:
        stride = wires.shape[1]
    nrec = wires.numel() // stride
    if len(slots) != len(weights) or not slots:
        raise ValueError("one weight per slot, at least one")
    if min(slots) < 0 or max(slots) >= nrec:
        raise ValueError(f"slots must index the {nrec} records")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an out tensor")
        out = torch.empty(n, dtype=torch.float32, device=wires.device)
    elif out.device != wires.device or out.dtype != torch.float32 or not out.is_contiguous() or out.numel() != n:
        raise ValueError(f"out must be a contiguous fp32 tensor of {n} elements on {wires.device}")
    m = len(slots)
    sl = (ctypes.c_int32 * m)(*[int(v) for v in slots])
    wt = (ctypes.c_float * m)(*[float(v) for v in weights])
    call("flc_stacked_fold_wires", _p(wires), stride, ctypes.cast(sl, ctypes.c_void_p), ctypes.cast(wt, ctypes.c_void_p),
         m, n, k, levels, int(accumulate), _p(out), _stream(out.device))
    return out


# -------------------------------------------------------------------------------------- adaptive random
ADAPTIVE_ERRORS = {1: "probabilities contain NaN", 2: "probabilities do not sum to 1"}


def adaptive_prepare(x: torch.Tensor) -> torch.Tensor:
    """First half of the adaptive random compressor (compressors.py:297-301): S = sum|x| in numpy's order,
    p = |x| / S, and the speculated runs of the fp64 cumsum.  Returns numpy's check as a device int32:
    0 = ok, 1 = NaN in p, 2 = p does not sum to 1 (see ADAPTIVE_ERRORS).  No uniform is consumed.  A float64 x
    runs the float64 form (S and p in fp64, flc_adaptive_prepare_f64)."""
    f64 = isinstance(x, torch.Tensor) and x.dtype == torch.float64
    x = (_dev_f64(x) if f64 else _dev_f32(x)).reshape(-1)
    n = x.numel()
    if n == 0:
        raise ValueError("'a' cannot be empty unless no samples are taken")
    status = torch.empty(1, dtype=torch.int32, device=x.device)
    ws = workspace(x.device, _ws_size(x.device, "flc_adaptive_workspace_size", n), "adaptive")
    call("flc_adaptive_prepare_f64" if f64 else "flc_adaptive_prepare", _p(x), n, _p(status), _p(ws), ws.numel(),
         _stream(x.device))
    return status


def adaptive_select(x: torch.Tensor, u: float, out: Optional[torch.Tensor] = None
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Second half, after :func:`adaptive_prepare` on the same stream: the exact sequential cdf,
    ``searchsorted(u, side='right')`` and the dense output (zeros, out[ind] = x[ind]).
    Returns (out, index as a device int64)."""
    f64 = isinstance(x, torch.Tensor) and x.dtype == torch.float64
    x = (_dev_f64(x) if f64 else _dev_f32(x)).reshape(-1)
    n = x.numel()
    if out is None:
        out = torch.empty(n, dtype=x.dtype, device=x.device)
    index = torch.empty(1, dtype=torch.int64, device=x.device)
    ws = workspace(x.device, _ws_size(x.device, "flc_adaptive_workspace_size", n), "adaptive")
    call("flc_adaptive_select_f64" if f64 else "flc_adaptive_select", _p(x), n, float(u), _p(index), _p(out), _p(ws),
         ws.numel(), _stream(x.device))
    return out, index


def adaptive_stats(x: torch.Tensor) -> dict:
    """Diagnostics of the last :func:`adaptive_select` on x's workspace (host sync): special chunks, special maps
    taken, chunks re-run sequentially, and whether the exact sequential chain ran instead."""
    x = x.reshape(-1)
    n = x.numel()
    ws = workspace(x.device, _ws_size(x.device, "flc_adaptive_workspace_size", n), "adaptive")
    st = torch.empty(4, dtype=torch.int32, device=x.device)
    call("flc_adaptive_stats", _p(ws), ws.numel(), n, _p(st), _stream(x.device))
    s = [int(v) for v in st.cpu()]
    return {"special": s[0], "taken": s[1], "reruns": s[2], "sequential": s[3]}


# ------------------------------------------------------------------------------------------------- misc
def copy(x: torch.Tensor) -> torch.Tensor:
    x = _dev_f32(x)
    out = torch.empty_like(x)
    call("flc_copy", _p(x), x.numel(), _p(out), _stream(x.device))
    return out


def scale_div(x: torch.Tensor, p: float) -> torch.Tensor:
    x = _dev_f32(x)
    out = torch.empty_like(x)
    call("flc_scale_div", _p(x), x.numel(), p, _p(out), _stream(x.device))
    return out


def randk_indices(n: int, k: int, seed: int, counter: int, device: torch.device) -> torch.Tensor:
    """Rand-K's index set in philox mode, on the device: the k largest of n Philox keys (flc_randk_keys + the top-k
    encoder), int32 ascending.  k >= n gives every index (the reference's ``S[:K]`` of a full permutation)."""
    if k >= n:
        return torch.arange(n, dtype=torch.int32, device=device)
    if k <= 0:
        return torch.empty(0, dtype=torch.int32, device=device)
    keys = torch.empty(n, dtype=torch.float32, device=device)
    call("flc_randk_keys", n, seed, counter, _p(keys), _stream(device))
    idx, _ = topk_encode(keys, k)
    return idx


def randk_apply(x: torch.Tensor, idx: torch.Tensor, scale: float) -> torch.Tensor:
    x = _dev_f32(x).reshape(-1)
    out = torch.empty_like(x)
    call("flc_randk_apply", _p(x), x.numel(), _p(idx), idx.numel(), scale, _p(out), _stream(x.device))
    return out


def weighted_sum(dst: torch.Tensor, srcs: Sequence[torch.Tensor], weights: Sequence[float], init_mode: int,
                 beta: float = 0.0) -> torch.Tensor:
    """dst = {dst*beta | 0 | dst} then dst = fmaf(w_m, src_m, dst) for each message in order."""
    import ctypes

    f64 = dst.dtype == torch.float64  # float64 models: the fold in fp64, the weights kept double (flc_weighted_sum_f64)
    if dst.device.type != "cuda" or dst.dtype not in (torch.float32, torch.float64) or not dst.is_contiguous():
        raise TypeError("dst must be a contiguous fp32 or fp64 HIP tensor")
    n = dst.numel()
    srcs = [(_dev_f64 if f64 else _dev_f32)(s, "src") for s in srcs]
    for s in srcs:
        if s.numel() != n:
            raise ValueError("every source must have dst's number of elements")
    ptrs = (ctypes.c_void_p * max(len(srcs), 1))(*[s.data_ptr() for s in srcs])
    ws = ((ctypes.c_double if f64 else ctypes.c_float) * max(len(srcs), 1))(*[float(w) for w in weights])
    call("flc_weighted_sum_f64" if f64 else "flc_weighted_sum", ctypes.cast(ptrs, ctypes.c_void_p),
         ctypes.cast(ws, ctypes.c_void_p), len(srcs), n, init_mode, float(beta), _p(dst), _stream(dst.device))
    return dst


MODEL_FOLD_MAX_SRC = 16


_MODEL_FOLD_OP: list = []


def _model_fold_op():
    """torch.ops.flcodec.model_fold_ when libflcodec_torch.so is built (the same C-ABI call, its per-tensor checks in
    C++), else None (the ctypes path below)."""
    if not _MODEL_FOLD_OP:
        op = None
        try:
            from . import load_torch_ops

            load_torch_ops()
            op = torch.ops.flcodec.model_fold_
        except (ImportError, OSError, RuntimeError, AttributeError):
            op = None
        _MODEL_FOLD_OP.append(op)
    return _MODEL_FOLD_OP[0]


_PYFOLD: list = []


def _pyfold():
    """fl_sim_amd._flcfold.model_fold (csrc/pyfold.cpp: the fold on Python lists of tensors, no dispatcher boxing,
    more than 16 messages in chained launches) when built, else None."""
    if not _PYFOLD:
        try:
            from . import _flcfold

            _PYFOLD.append(_flcfold.model_fold)
        except ImportError:
            _PYFOLD.append(None)
    return _PYFOLD[0]


_PYSRV: list = []


def _pysrv():
    """fl_sim_amd._flcfold.server_fold (csrc/pyfold.cpp: flc_model_fold_server on Python lists of tensors, at most 16
    messages) when built, else None."""
    if not _PYSRV:
        try:
            from . import _flcfold

            _PYSRV.append(_flcfold.server_fold)
        except (ImportError, AttributeError):
            _PYSRV.append(None)
    return _PYSRV[0]


_PYPAIR: list = []


def _pypair():
    """fl_sim_amd._flcfold.avg_and_gradients (csrc/pyfold.cpp: flc_avg_and_gradients on Python lists of tensors and
    message mappings) when built, else None."""
    if not _PYPAIR:
        try:
            from . import _flcfold

            _PYPAIR.append(_flcfold.avg_and_gradients)
        except (ImportError, AttributeError):
            _PYPAIR.append(None)
    return _PYPAIR[0]


_PYDELTA: list = []
_PYFLAT: list = []
_PYBATCH: list = []
_PYRECS: list = []


def _pyrecs():
    """fl_sim_amd._flcfold.fold_records (flc_fedopt_fold_records on Python lists, one C call) when built, else None."""
    if not _PYRECS:
        try:
            from . import _flcfold

            _PYRECS.append(_flcfold.fold_records)
        except (ImportError, AttributeError):
            _PYRECS.append(None)
    return _PYRECS[0]


def _pyflat():
    """fl_sim_amd._flcfold.delta_flat (a new flat delta, flc_delta_flatten, one C call) when built, else None."""
    if not _PYFLAT:
        try:
            from . import _flcfold

            _PYFLAT.append(_flcfold.delta_flat)
        except (ImportError, AttributeError):
            _PYFLAT.append(None)
    return _PYFLAT[0]


def _pybatch():
    """fl_sim_amd._flcfold.stacked_records_batch (the batched stacked encode into a record block and the batched
    send counts, one C call) when built, else None."""
    if not _PYBATCH:
        try:
            from . import _flcfold

            _PYBATCH.append(_flcfold.stacked_records_batch)
        except (ImportError, AttributeError):
            _PYBATCH.append(None)
    return _PYBATCH[0]


def _pydelta():
    """fl_sim_amd._flcfold.stacked_delta_record (csrc/pyfold.cpp: the delta-fused stacked encode into a wire record and
    the send count, one C call on Python lists of tensors) when built, else None."""
    if not _PYDELTA:
        try:
            from . import _flcfold

            _PYDELTA.append(_flcfold.stacked_delta_record)
        except (ImportError, AttributeError):
            _PYDELTA.append(None)
    return _PYDELTA[0]


def model_fold_server(theta: Sequence[torch.Tensor], aux: Sequence[torch.Tensor],
                      srcs: Sequence[Sequence[torch.Tensor]], weights: Sequence[float], kind: str, fold: bool = True,
                      init_mode: int = 0, inertia: float = 0.0, c: float = 0.0) -> None:
    """FedDyn's / pFedMe's server update of a whole model in one launch (flc_model_fold_server): ``kind`` "feddyn"
    (aux = h; c = -mu / num_clients) or "pfedme" (aux = the saved model when ``fold`` is False; c = beta).  ``srcs[m]``
    is message m's tensor list, at most 16 messages; every tensor a contiguous fp32 tensor on theta's device."""
    import ctypes

    nt, ns = len(theta), len(srcs)
    if ns > MODEL_FOLD_MAX_SRC:
        raise ValueError(f"model_fold_server takes at most {MODEL_FOLD_MAX_SRC} messages")
    if len(aux) != nt or len(weights) != ns or any(len(m) != nt for m in srcs):
        raise ValueError("one aux tensor per model tensor, one weight per message, one tensor per model tensor each")
    if nt == 0:
        return
    f32, dev = torch.float32, theta[0].get_device()
    sizes = [t.numel() for t in theta]

    def ptrs(ts):
        out = []
        for t, n in zip(ts, sizes):
            if not (t.is_cuda and t.dtype is f32 and t.is_contiguous() and t.get_device() == dev and t.numel() == n):
                raise TypeError("model_fold_server: contiguous fp32 HIP tensors of the model's sizes on one device")
            out.append(t.data_ptr())
        return out

    sp = [q for m in srcs for q in ptrs(m)]
    P = ctypes.c_void_p
    vp = lambda a: ctypes.cast(a, P)  # noqa: E731
    call("flc_model_fold_server", vp((P * nt)(*ptrs(theta))), vp((P * nt)(*ptrs(aux))), vp((P * max(len(sp), 1))(*sp)),
         vp((ctypes.c_float * max(ns, 1))(*[float(w) for w in weights])), ns, vp((ctypes.c_int64 * nt)(*sizes)), nt,
         {"feddyn": _lib.FLC_SRV_FEDDYN, "pfedme": _lib.FLC_SRV_PFEDME}[kind], int(bool(fold)), int(init_mode),
         float(inertia), float(c), _stream(theta[0].device))


def model_fold(dsts: Sequence[torch.Tensor], srcs: Sequence[Sequence[torch.Tensor]], weights: Sequence[float],
               init_mode: int, beta: float = 0.0, theta: Optional[Sequence[torch.Tensor]] = None,
               v: Optional[Sequence[torch.Tensor]] = None, opt: str = "avg", lr: float = 1.0, beta2: float = 0.0,
               tau: float = 0.0) -> None:
    """A whole model in one launch (flc_model_fold): per tensor t, ``weighted_sum(dsts[t], [s[t] for s in srcs],
    weights, init_mode, beta)`` and, with ``theta``, ``fedopt_step(theta[t], dsts[t], v[t], opt, lr, beta2, tau)``.
    ``srcs[m]`` is message m's list of tensors (all on the dsts' device); at most 16 messages.  The checks are one
    lean pass per tensor: a model update is ~100 tensors, and per-tensor Python costs more than the kernel."""
    import ctypes

    nt, ns = len(dsts), len(srcs)
    pf = _pyfold()
    if pf is not None:  # every tensor checked in C before anything is launched; > 16 messages chained
        pf(dsts, srcs, None, weights, int(init_mode), float(beta), theta, v, _lib.FLC_OPT[opt], float(lr), float(beta2),
           float(tau))
        return
    if ns > MODEL_FOLD_MAX_SRC:
        raise ValueError(f"model_fold takes at most {MODEL_FOLD_MAX_SRC} messages")
    if nt == 0:
        return
    op = _model_fold_op()
    if op is not None:  # the checks and the pointer tables in C++ (torch_ops.cpp): one dispatcher call
        if any(len(msg) != nt for msg in srcs):
            raise ValueError("every message has one tensor per model tensor")
        if len(weights) != ns:
            raise ValueError("one weight per message")
        op(list(dsts), [t for msg in srcs for t in msg], [float(w) for w in weights], int(init_mode), float(beta),
           [] if theta is None else list(theta), [] if v is None else list(v), _lib.FLC_OPT[opt], float(lr),
           float(beta2), float(tau))
        return
    f32 = torch.float32
    dev = dsts[0].get_device()

    def ptrs(ts, what):
        out = []
        for t in ts:
            if not (t.is_cuda and t.dtype is f32 and t.is_contiguous() and t.get_device() == dev):
                raise TypeError(f"{what} tensors must be contiguous fp32 HIP tensors on one device")
            out.append(t.data_ptr())
        return out

    if len(weights) != ns:
        raise ValueError("one weight per message")
    sizes = [t.numel() for t in dsts]
    for what, ts in (("theta", theta), ("v", v)):
        if ts is not None and (len(ts) != nt or any(t.numel() != n for t, n in zip(ts, sizes))):
            raise ValueError(f"{what} must have one tensor per model tensor, of the model tensors' sizes")
    dp = ptrs(dsts, "model")
    sp = []
    for msg in srcs:
        if len(msg) != nt:
            raise ValueError("every message has one tensor per model tensor")
        for a, n in zip(msg, sizes):
            if a.numel() != n:
                raise ValueError("message tensors must match the model tensors' sizes")
        sp.extend(ptrs(msg, "message"))
    P = ctypes.c_void_p
    vp = lambda a: ctypes.cast(a, P)  # noqa: E731
    call("flc_model_fold", vp((P * nt)(*dp)), vp((P * max(len(sp), 1))(*sp)),
         vp((ctypes.c_float * max(ns, 1))(*weights)), ns, vp((ctypes.c_int64 * nt)(*sizes)), nt, int(init_mode),
         float(beta), None if theta is None else vp((P * nt)(*ptrs(theta, "model"))),
         None if v is None else vp((P * nt)(*ptrs(v, "model"))), _lib.FLC_OPT[opt], float(lr), float(beta2),
         float(tau), torch.cuda.current_stream(dev).cuda_stream)


def fedopt_step(theta: torch.Tensor, delta: torch.Tensor, v: Optional[torch.Tensor], opt: str, lr: float,
                beta2: float, tau: float) -> None:
    dt = theta.dtype
    for t, name in ((theta, "theta"), (delta, "delta"), (v, "v")):
        if t is None:
            continue
        if t.device.type != "cuda" or t.dtype != dt or dt not in (torch.float32, torch.float64) or not t.is_contiguous():
            raise TypeError(f"{name} must be a contiguous HIP tensor of theta's dtype (fp32 or fp64)")
        if t.numel() != theta.numel():
            raise ValueError("theta, delta and v must have the same number of elements")
    call("flc_fedopt_step_f64" if dt == torch.float64 else "flc_fedopt_step", _p(theta), _p(delta), _p(v),
         theta.numel(), _lib.FLC_OPT[opt], float(lr), float(beta2), float(tau), _stream(theta.device))


def feddr_combine(theta: torch.Tensor, y: torch.Tensor, x_til: torch.Tensor, alpha: float, cx: float, cy: float,
                  prox: int, prox_c: float) -> None:
    """y = fmaf(alpha, theta - y, y); theta = prox(cx * x_til + cy * y), in place (flc_feddr_combine)."""
    dt = theta.dtype
    for t, name in ((theta, "theta"), (y, "y"), (x_til, "x_til")):
        if t.device.type != "cuda" or t.dtype != dt or dt not in (torch.float32, torch.float64) or not t.is_contiguous():
            raise TypeError(f"{name} must be a contiguous HIP tensor of theta's dtype (fp32 or fp64)")
        if t.numel() != theta.numel():
            raise ValueError("theta, y and x_til must have the same number of elements")
    call("flc_feddr_combine_f64" if dt == torch.float64 else "flc_feddr_combine", _p(theta), _p(y), _p(x_til),
         theta.numel(), float(alpha), float(cx), float(cy), int(prox), float(prox_c), _stream(theta.device))


def delta_flatten(local_params: Sequence[torch.Tensor], global_params: Sequence[torch.Tensor],
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The flat client delta ``cat([l - g for l, g in zip(local, global)])`` in one pass (flc_delta_flatten):
    FedOptClient.communicate's clone + ``add_(alpha=-1)`` (_fedopt.py:294-297) fused with the flatten the codec
    input needs.  Returns ``out`` (allocated when None)."""
    import ctypes

    ls = [_dev_f32(t, "local") for t in local_params]
    gs = [_dev_f32(t, "global") for t in global_params]
    if len(ls) != len(gs):
        raise ValueError("one global tensor per local tensor")
    for a, b in zip(ls, gs):
        if a.numel() != b.numel() or a.device != b.device:
            raise ValueError("local and global tensors must match in size and device")
    total = sum(t.numel() for t in ls)
    dev = ls[0].device if ls else (out.device if out is not None else torch.device("cuda"))
    if out is None:
        out = torch.empty(total, dtype=torch.float32, device=dev)
    elif out.device.type != "cuda" or out.dtype != torch.float32 or not out.is_contiguous() or out.numel() != total:
        raise ValueError(f"out must be a contiguous fp32 HIP tensor of {total} elements")
    m = max(len(ls), 1)
    lp = (ctypes.c_void_p * m)(*[t.data_ptr() for t in ls])
    gp = (ctypes.c_void_p * m)(*[t.data_ptr() for t in gs])
    sz = (ctypes.c_int64 * m)(*[t.numel() for t in ls])
    call("flc_delta_flatten", ctypes.cast(lp, ctypes.c_void_p), ctypes.cast(gp, ctypes.c_void_p),
         ctypes.cast(sz, ctypes.c_void_p), len(ls), _p(out), _stream(dev))
    return out


# ---------------------------------------------------------------------------------------- float64 inputs
# The reference runs every compressor on whatever dtype x has (compressors.py:267-410); these are the float64 forms
# (f64.hip): a float64 HIP vector in, a float64 HIP vector out.  Uniforms as for float32 (compat_u: one double per
# consumer in index order, else Philox at the element's index).
def _dev_f64(x: torch.Tensor, name: str = "x") -> torch.Tensor:
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
        raise TypeError(f"{name} must be a torch tensor on a HIP device")
    if x.dtype != torch.float64:
        raise TypeError(f"{name} must be float64 (got {x.dtype})")
    x = x.reshape(-1)
    if not x.is_contiguous() or x.data_ptr() % 16 != 0:
        x = x.contiguous().clone()
    return x


def _ws64(x: torch.Tensor, k: int = 0) -> torch.Tensor:
    return workspace(x.device, _ws_size(x.device, "flc_f64_workspace_size", x.numel(), int(k)), "f64")


def copy_f64(x: torch.Tensor) -> torch.Tensor:
    x = _dev_f64(x)
    out = torch.empty_like(x)
    call("flc_copy_f64", _p(x), x.numel(), _p(out), _stream(x.device))
    return out


def scale_div_f64(x: torch.Tensor, p: float) -> torch.Tensor:
    x = _dev_f64(x)
    out = torch.empty_like(x)
    call("flc_scale_div_f64", _p(x), x.numel(), float(p), _p(out), _stream(x.device))
    return out


def randk_apply_f64(x: torch.Tensor, idx: torch.Tensor, scale: float) -> torch.Tensor:
    x = _dev_f64(x)
    idx = idx.to(device=x.device, dtype=torch.int32).contiguous()
    out = torch.empty_like(x)
    call("flc_randk_apply_f64", _p(x), x.numel(), _p(idx), idx.numel(), float(scale), _p(out), _stream(x.device))
    return out


def count_consumers_f64(x: torch.Tensor, norm: Optional[torch.Tensor]) -> torch.Tensor:
    """Device int64 scalar: the uniforms the reference draws (natural: norm None, x != 0; dithering: with the norm)."""
    x = _dev_f64(x)
    out = torch.empty(1, dtype=torch.int64, device=x.device)
    ws = _ws64(x)
    call("flc_count_consumers_f64", _p(x), x.numel(), _p(norm), _p(out), _p(ws), ws.numel(), _stream(x.device))
    return out


def natural_f64(x: torch.Tensor, seed: int = 0, counter: int = 0, compat_u: Optional[torch.Tensor] = None,
                want_codes: bool = False) -> Tuple[Optional[torch.Tensor], torch.Tensor]:
    """Natural compression of a float64 vector: (codes or None, decoded float64 vector)."""
    x = _dev_f64(x)
    n = x.numel()
    codes = torch.empty(n, dtype=torch.int16, device=x.device) if want_codes else None
    out = torch.empty_like(x)
    ws = _ws64(x)
    call("flc_natural_f64", _p(x), n, seed, counter, _p(compat_u), _p(codes), _p(out), _p(ws), ws.numel(),
         _stream(x.device))
    return codes, out


def natural_decode_f64(codes: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.empty(n, dtype=torch.float64, device=codes.device)
    call("flc_natural_decode_f64", _p(codes), n, _p(out), _stream(out.device))
    return out


def quant_norm_f64(x: torch.Tensor, p: float = math.inf) -> torch.Tensor:
    x = _dev_f64(x)
    pk = _lib.FLC_NORM_INF if math.isinf(p) else (_lib.FLC_NORM_L2 if p == 2 else None)
    if pk is None:
        raise ValueError(f"p must be inf or 2 (got {p})")
    norm = torch.empty(1, dtype=torch.float64, device=x.device)
    ws = _ws64(x)
    call("flc_quant_norm_f64", _p(x), x.numel(), pk, _p(norm), _p(ws), ws.numel(), _stream(x.device))
    return norm


def quant_f64(x: torch.Tensor, kind: int, levels: int, norm: torch.Tensor, seed: int = 0, counter: int = 0,
              compat_u: Optional[torch.Tensor] = None, want_codes: bool = False, want_nnz: bool = False):
    """Standard / natural dithering of a float64 vector with the given float64 norm (a 1-element device tensor):
    (8-bit codes or None, decoded float64 vector, nnz or None)."""
    x = _dev_f64(x)
    n = x.numel()
    if norm.dtype != torch.float64 or norm.device != x.device:
        raise TypeError("norm must be a float64 tensor on x's device")
    if compat_u is not None and compat_u.dtype != torch.float64:
        raise TypeError("compat_u must be float64")
    codes = torch.empty(n, dtype=torch.uint8, device=x.device) if want_codes else None
    nnz = torch.empty(1, dtype=torch.int64, device=x.device) if want_nnz else None
    out = torch.empty_like(x)
    ws = _ws64(x)
    call("flc_quant_f64", _p(x), n, kind, levels, _p(norm), seed, counter, _p(compat_u), _p(codes), _p(out), _p(nnz),
         _p(ws), ws.numel(), _stream(x.device))
    return codes, out, nnz


def quant_decode_f64(codes: torch.Tensor, n: int, kind: int, levels: int, norm: torch.Tensor) -> torch.Tensor:
    out = torch.empty(n, dtype=torch.float64, device=codes.device)
    call("flc_quant_decode_f64", _p(codes), n, kind, levels, _p(norm), _p(out), _stream(out.device))
    return out


def topk_dense_f64(x: torch.Tensor, k: int) -> torch.Tensor:
    """out = x on the k largest elements (ties: the highest indices), +0 elsewhere; 0 < k < n."""
    x = _dev_f64(x)
    out = torch.empty_like(x)
    ws = _ws64(x, k)
    call("flc_topk_dense_f64", _p(x), x.numel(), int(k), _p(out), _p(ws), ws.numel(), _stream(x.device))
    _after_encode(x.device, ("f64",))
    return out
