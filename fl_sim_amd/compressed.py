"""The codec's call site: a FedOpt round whose client messages carry a compressed delta.

The reference never calls its compressors (``.coveragerc:16-17``; the only caller is
``test/test_compressors.py:12-15``), so the call site is new.  Its meaning is fixed by the round fixtures
(``tests/golden/gen_golden.py`` ``gen_round``), composed from the reference's own pieces:

* client — ``FedOptClient.communicate`` (``_fedopt.py:295-308``) forms ``delta_j = θ_local_j − θ_global_j``; the
  flattened delta goes through ``Compressor.compressVector`` (``compressors.py:267-410``): one compressor, or the
  stacked pipeline TopK then standard dithering (p = ∞) of the K-sparse result; the decoded vector, reshaped to the
  model's tensors, is the message's ``delta_parameters``;
* server — ``FedOptServer.update`` (``_fedopt.py:196-240``) folds the round.

What runs here instead:

* :class:`CompressedFedOptClientMixin` — ``communicate`` forms the delta on the device.  With the stacked pipeline the
  message carries the client's packed wire record (``flc_stacked_wire_layout``: 5 B per kept entry + tile pointers)
  instead of the dense delta; in philox mode the delta is formed inside the encoder's read
  (``flc_stacked_encode_delta``), in compat mode the pipeline is composed from the top-k encode and the dithering
  encode of the kept values with the interpreter's ``random`` stream, exactly as the reference consumes it.  Any other
  compressor runs through the drop-in ``Compressor`` on the device and the message carries the decoded delta.
  Either way ``delta_parameters`` is a :class:`CompressedDelta`: a sequence of per-tensor tensors that decodes itself
  on first access, so any server — the reference's own ``update`` included — reads it unchanged.
* ``aggregation.fedopt_update`` (and :class:`~fl_sim_amd.aggregation.FedOptUpdateMixin`) recognises a round of stacked
  records and runs :func:`fold_records`: ONE launch per 64 clients decodes every record, folds it into δ in message
  order and applies the server optimiser's step (``flc_fedopt_fold_records``) — the records are read once, δ, θ (and
  v) read and written once; bit-identical to decoding each record and running the reference's update.

The compressors' send statistics advance as ``compressVector`` advances them (``compressors.py:406-408``), per stage.
"""

from __future__ import annotations

import collections.abc as _abc
import ctypes
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib, codec
from ._lib import FLC_NORM_INF, FLC_Q_STANDARD_DITHER
from .compressors import Compressor, CompressorType


_MSG_CLS: list = []


def client_message_class():
    """The reference's ``ClientMessage`` (nodes.py:1537-1557) when ``fl_sim`` is importable (``Server._update``
    asserts the type, nodes.py:767-770), else a dict subclass with the same constructor.  Looked up once per process
    (a failing import costs ~80 us, and ``communicate`` runs once per client per round)."""
    if not _MSG_CLS:
        try:
            from fl_sim.nodes import ClientMessage as ref_cls  # type: ignore
        except Exception:  # fl_sim absent (or its dependencies: torch_ecg, ...)
            ref_cls = ClientMessage
        _MSG_CLS.append(ref_cls)
    return _MSG_CLS[0]


class ClientMessage(dict):
    """Stand-in for the reference's ``ClientMessage`` (nodes.py:1537-1557) when ``fl_sim`` is not importable."""

    __name__ = "ClientMessage"

    def __init__(self, client_id: int, train_samples: int, metrics: dict, **kwargs) -> None:
        super().__init__(client_id=client_id, train_samples=train_samples, metrics=metrics, **kwargs)


class CompressedDelta(_abc.Sequence):
    """A client's compressed model delta as its message carries it.

    ``kind == "stacked"``: the packed wire record of the stacked codec (top-k ascending int32 indices, 8-bit
    sign | level codes, the kept set's norm, tile pointers); ``kind == "dense"``: the decoded flat delta.  Indexing
    gives tensor ``j`` of the model's shapes (the decoded values, one flat decode on first access), so code written for
    a list of delta tensors reads it unchanged."""

    def __init__(self, shapes: Sequence[torch.Size], device: torch.device, n: int, *, record=None, k: int = 0,
                 levels: int = 0, flat: Optional[torch.Tensor] = None, batch: Optional["_Batch"] = None):
        self.shapes = [torch.Size(s) for s in shapes]
        self.device = device
        self.n = int(n)
        self._record, self.k, self.levels = record, int(k), int(levels)
        self._batch = batch  # (a deferred encode: the record is made by the batch's launch on first access)
        self.kind = "stacked" if record is not None or batch is not None else "dense"
        self._flat = flat
        self._views: Optional[List[torch.Tensor]] = None

    @property
    def record(self) -> Optional[torch.Tensor]:
        """The packed wire record (stacked), or None (dense)."""
        if self._batch is not None:
            self._batch.run()
        return self._record

    def __getstate__(self):
        """A copied or pickled message carries its record (a deferred encode runs first)."""
        if self._batch is not None:
            self._batch.run()
        d = self.__dict__.copy()
        d["_batch"] = None
        return d

    @property
    def nbytes(self) -> int:
        """Bytes the message carries for the delta (the wire record, or the dense fp32 vector)."""
        return int(self.record.numel()) if self.record is not None else 4 * self.n

    def flat(self) -> torch.Tensor:
        """The decoded flat delta (stacked: flc_stacked_decode_tiled of the record, once)."""
        if self._flat is None:
            self._flat = codec.stacked_decode(codec.wire_packet(self.record, self.n, self.k, self.levels))
        return self._flat

    def tensors(self) -> List[torch.Tensor]:
        if self._views is None:
            f, out, off = self.flat(), [], 0
            for s in self.shapes:
                m = s.numel()
                out.append(f[off:off + m].view(s))
                off += m
            self._views = out
        return self._views

    def __len__(self) -> int:
        return len(self.shapes)

    def __getitem__(self, j):
        return self.tensors()[j]

    def __iter__(self):
        return iter(self.tensors())


def stacked_pipeline(compressors: Sequence[Compressor]) -> Optional[Tuple[int, int]]:
    """(K, levels) when ``compressors`` is the stacked pipeline the packed wire carries: a TopK compressor, then a
    float32 standard-dithering compressor with p = ∞ and 1..127 levels; else None."""
    if len(compressors) != 2:
        return None
    tk, sd = compressors
    if not (isinstance(tk, Compressor) and isinstance(sd, Compressor)):
        return None
    if tk.compressorType != CompressorType.TOPK_COMPRESSOR:
        return None
    if sd.compressorType != CompressorType.STANDARD_DITHERING_FP32 or not math.isinf(sd.p) or not 1 <= sd.s <= 127:
        return None
    return int(tk.K), int(sd.s)


def _ptrs(ts: Sequence[torch.Tensor]):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def _fp32_on(ts: Sequence[torch.Tensor], dev: torch.device) -> List[torch.Tensor]:
    out = []
    for t in ts:
        t = t.detach()
        if t.device != dev:
            t = t.to(dev)
        if t.dtype != torch.float32 or not t.is_contiguous() or t.data_ptr() % 4:
            t = t.contiguous().float()
        out.append(t)
    return out


def _norm_stage_send(sd: Compressor, norm: torch.Tensor) -> float:
    """The norm compressor's pass over the one-element norm vector (compressors.py:334-337) and the send count it
    contributes; an identical norm compressor (the reference's usual one) is advanced without reading the norm back."""
    nc = sd.vectorNormCompressor
    if _identical(nc):
        nc._finish(1, 1)
    else:
        nc.compressVector(np.array([np.float32(norm.item())]))
    return nc.last_need_to_send_advance


def compress_delta(local: Sequence[torch.Tensor], cached: Sequence[torch.Tensor],
                   compressors: Sequence[Compressor]) -> CompressedDelta:
    """The client's compressed delta ``compressors(cat(local − cached))`` (see the module docstring); every compressor's
    RNG stream and send statistics advance as its own ``compressVector`` call would advance them."""
    local = list(local)
    dev = local[0].device if local[0].is_cuda else torch.device("cuda", torch.cuda.current_device())
    shapes = [t.shape for t in local]
    n = sum(t.numel() for t in local)
    pipe = stacked_pipeline(compressors)
    seed_ctr = None
    if pipe is not None and 0 < pipe[0] < n and compressors[1].rng_mode == "philox":
        # the common case in one C call, the tensors as they are (model parameters on the device): the record and the
        # send count made by _flcfold.stacked_delta_record; a tensor it does not take (host-resident, not fp32 or not
        # contiguous) falls through to the converted call below with the same Philox (seed, counter)
        seed_ctr = compressors[1].philox.next()
        if DEFER_ENCODE and n <= _DEFER_MAX_N and _identical(compressors[1].vectorNormCompressor):
            r = _deferred(local, cached, shapes, n, pipe[0], pipe[1], compressors[0], compressors[1], dev, seed_ctr)
            if r is not None:
                return r
        r = _stacked_fast(local, cached, shapes, n, pipe[0], pipe[1], compressors[0], compressors[1], dev, seed_ctr)
        if r is not None:
            return r
    out = None
    if pipe is None or not 0 < pipe[0] < n:
        snap = codec._pyflat()
        if snap is not None:
            try:  # the flat delta in one C call (the tensors as they are: contiguous fp32 on one device)
                out = snap(local, cached)
            except TypeError:
                pass
            if out is not None and out.device != dev:
                out = None
    if out is None:
        ls, gs = _fp32_on(local, dev), _fp32_on(cached, dev)
        if pipe is not None and 0 < pipe[0] < n:
            return _stacked(ls, gs, shapes, n, pipe[0], pipe[1], compressors[0], compressors[1], dev, seed_ctr)
        out = codec.delta_flatten(ls, gs)
    for comp in compressors:  # the drop-in compressors on the device, in order
        out = comp.compressVector(out)
    return CompressedDelta(shapes, dev, n, flat=out)


# Deferred encodes (philox mode, the stacked pipeline, an identical norm compressor, models up to 16 M parameters).
# A model-sized encode is all fixed latency on the GPU — ~44 us per message at configs[0] (417,482 parameters), most of
# it the persistent select's grid exchanges — so a round's messages are encoded together: `communicate` flattens the
# client's delta (a snapshot: the model may change before the encode runs) and fixes its Philox (seed, counter) and
# send-count slot, and the first access to any of the round's records — or to a statistic of their compressors —
# encodes them all in one launch (flc_stacked_encode_batch: each client's select on its share of the CUs, records
# bit-identical to the per-message encodes) and counts their dithering stages' nonzero inputs in one more
# (flc_count_nonzero_at_batch).  FLC_DEFER_ENCODE=0 encodes every message when it is made (the one-C-call form).
DEFER_ENCODE = os.environ.get("FLC_DEFER_ENCODE", "1") != "0"
_DEFER_MAX_N = 1 << 24
_DEFER_MAX_PENDING = 64
_DEFER_MAX_BATCHES = 16


class _Batch:
    """The waiting messages of one (device, n, k, levels, counter)."""

    def __init__(self, key):
        self.key = key
        self.items = []  # (CompressedDelta, flat delta, seed, count slot, dithering compressor, stream, its handle)

    def run(self) -> None:
        if _PENDING.get(self.key) is self:
            del _PENDING[self.key]
        items, self.items = self.items, []
        if not items:
            return
        try:
            self._encode(items)
        except BaseException:
            self.items = items + self.items  # (left pending: the next access tries again and raises again)
            _PENDING.setdefault(self.key, self)
            raise

    def _encode(self, items) -> None:
        di, n, k, levels, counter = self.key
        dev = torch.device("cuda", di)
        with torch.cuda.device(dev):
            cur = torch.cuda.current_stream(dev)
            ch = cur.cuda_stream
            for st in {it[6]: it[5] for it in items if it[6] != ch}.values():  # (deltas flattened on other streams)
                cur.wait_stream(st)
            stride, off = codec.stacked_wire_layout(n, k)
            C = len(items)
            recs = torch.empty(C, stride, dtype=torch.uint8, device=dev)
            flats = [it[1] for it in items]
            fast = codec._pybatch()
            if fast is not None:  # both launches in one C call
                ws = codec.workspace(dev, codec._ws_size(dev, "flc_stacked_encode_batch_workspace_size", n, k, C),
                                     "topk_batch")
                fast(flats, [it[2] for it in items], counter, k, levels, recs, [it[3] for it in items], ws)
            else:
                codec.stacked_encode_batch(flats, k, levels, seeds=[it[2] for it in items], counter=counter,
                                           wires=recs)
                P = ctypes.c_void_p * C
                _lib.call("flc_count_nonzero_at_batch", P(*[f.data_ptr() for f in flats]),
                          P(*[recs[c].data_ptr() + off["idx"] for c in range(C)]), C, n, k,
                          P(*[it[3].data_ptr() for it in items]), codec._stream(dev))
            codec._after_encode(dev)
            for (d, flat, _, _, sd, _, sh), r in zip(items, recs.unbind(0)):
                if sh != ch:
                    flat.record_stream(cur)
                    sd._note_slab_stream(cur)  # (the count was written on this stream, not the slot's own)
                d._record, d._batch = r, None


_PENDING: dict = {}


def _run_pending() -> None:
    """Every deferred encode now (before a compressor's pending send counts are read)."""
    for b in list(_PENDING.values()):
        b.run()


Compressor._before_read = staticmethod(_run_pending)


def _deferred(local, cached, shapes, n: int, K: int, s: int, tk: Compressor, sd: Compressor, dev,
              seed_ctr) -> Optional[CompressedDelta]:
    snap = codec._pyflat()
    try:
        flat = snap(local, cached) if snap is not None else codec.delta_flatten(local, cached)
    except TypeError:  # (host-resident, non-contiguous or non-fp32 tensors: converted first)
        flat = codec.delta_flatten(_fp32_on(local, dev), _fp32_on(cached, dev))
    if flat.device != dev:
        return None
    st = torch.cuda.current_stream(dev)
    cnt = sd._count_slot(dev, st)  # (before the batch is looked up: a full slab is read back, running the batches)
    key = (dev.index, n, K, s, seed_ctr[1])
    b = _PENDING.get(key)
    if b is None:
        b = _PENDING[key] = _Batch(key)
    d = CompressedDelta(shapes, dev, n, k=K, levels=s, batch=b)
    b.items.append((d, flat, seed_ctr[0], cnt, sd, st, st.cuda_stream))
    tk._finish(n, tk.K)
    base = _norm_stage_send(sd, None)
    sd._finish_pending(n, cnt, base, (1.0 + np.ceil(math.log2(sd.s))) / 32.0)  # compressors.py:365
    if len(b.items) >= _DEFER_MAX_PENDING:
        b.run()
    elif len(_PENDING) > _DEFER_MAX_BATCHES:  # (messages nobody reads: the waiting deltas stay bounded)
        _run_pending()
    return d


def _stacked_fast(local, cached, shapes, n: int, K: int, s: int, tk: Compressor, sd: Compressor, dev,
                  seed_ctr) -> Optional[CompressedDelta]:
    """The philox-mode stacked message in one C call (None: the extension is absent or a tensor needs converting)."""
    fast = codec._pydelta()
    if fast is None:
        return None
    stride, _ = codec.stacked_wire_layout(n, K)
    rec = torch.empty(stride, dtype=torch.uint8, device=dev)
    cnt = sd._count_slot(dev)
    ws = codec.workspace(dev, codec._ws_size(dev, "flc_stacked_encode_delta_workspace_size", n, K, len(local)), "topk")
    try:
        fast(local, cached, K, s, seed_ctr[0], seed_ctr[1], rec, cnt, ws)
    except TypeError:
        return None  # (nothing launched)
    codec._after_encode(dev)
    tk._finish(n, tk.K)
    nc = sd.vectorNormCompressor
    base = _norm_stage_send(sd, None if _identical(nc) else codec.wire_packet(rec, n, K, s).norm)
    sd._finish_pending(n, cnt, base, (1.0 + np.ceil(math.log2(sd.s))) / 32.0)  # compressors.py:365
    return CompressedDelta(shapes, dev, n, record=rec, k=K, levels=s)


def _identical(nc) -> bool:
    return isinstance(nc, Compressor) and nc.compressorType == CompressorType.IDENTICAL


def _stacked(ls, gs, shapes, n: int, K: int, s: int, tk: Compressor, sd: Compressor, dev,
             seed_ctr=None) -> CompressedDelta:
    stride, _ = codec.stacked_wire_layout(n, K)
    rec = torch.empty(stride, dtype=torch.uint8, device=dev)
    pk = codec.wire_packet(rec, n, K, s)
    per = (1.0 + np.ceil(math.log2(sd.s))) / 32.0  # compressors.py:365
    seed, ctr = seed_ctr if seed_ctr is not None else sd.philox.next()
    if sd.rng_mode == "philox":
        # the delta formed inside the encoder's read; the dithering stage's nonzero count stays on the device
        codec.stacked_encode_delta(ls, gs, K, s, seed, ctr, wire=rec)
        cnt = sd._count_slot(dev)
        _lib.call("flc_delta_count_nonzero_at", _ptrs(ls), _ptrs(gs),
                  (ctypes.c_int64 * len(ls))(*[t.numel() for t in ls]), len(ls), pk.idx.data_ptr(), K,
                  cnt.data_ptr(), codec._stream(dev))
        tk._finish(n, tk.K)
        base = _norm_stage_send(sd, pk.norm)
        sd._finish_pending(n, cnt, base, per)
        return CompressedDelta(shapes, dev, n, record=rec, k=K, levels=s)
    # compat: TopK (compressors.py:293-296), then standard dithering of the K-sparse vector (327-365) whose nonzero
    # elements, in index order, are the kept values: one random.random() per consuming kept value
    x = codec.delta_flatten(ls, gs)
    val = torch.empty(K, dtype=torch.float32, device=dev)
    ws = codec.workspace(dev, codec._ws_size(dev, "flc_topk_workspace_size", n, K), "topk")
    st = codec._stream(dev)
    _lib.call("flc_topk_encode_tiled", x.data_ptr(), n, K, pk.idx.data_ptr(), val.data_ptr(), pk.tiles.data_ptr(),
              ws.data_ptr(), ws.numel(), st)
    codec._after_encode(dev)
    tk._finish(n, tk.K)
    row = val.reshape(1, K)
    qws = codec.workspace(dev, codec._ws_size(dev, "flc_quant_workspace_size", 1, K), "quant")
    _lib.call("flc_quant_norm", row.data_ptr(), 1, K, FLC_NORM_INF, pk.norm.data_ptr(), qws.data_ptr(), qws.numel(), st)
    consumers = int(codec.count_consumers(row, pk.norm).item())
    u = sd._uniforms(consumers, dev)
    nnz = torch.empty(1, dtype=torch.int64, device=dev)
    _lib.call("flc_quant_encode", row.data_ptr(), 1, K, FLC_Q_STANDARD_DITHER, s, 8, pk.norm.data_ptr(), seed, ctr,
              u.data_ptr() if consumers else None, pk.codes.data_ptr(), nnz.data_ptr(), qws.data_ptr(), qws.numel(), st)
    base = _norm_stage_send(sd, pk.norm)
    nz = int(nnz.item())
    sd._finish(n, base + nz * per if nz else base)
    return CompressedDelta(shapes, dev, n, record=rec, k=K, levels=s)


def stacked_round(messages: Sequence, key: str = "delta_parameters") -> Optional[List[CompressedDelta]]:
    """The messages' compressed deltas when every one is a stacked record of one (n, k, levels), else None."""
    if not messages:
        return None
    ds = []
    for m in messages:
        d = m.get(key) if isinstance(m, dict) else None
        if not isinstance(d, CompressedDelta) or d.kind != "stacked":
            return None
        ds.append(d)
    d0 = ds[0]
    if any((d.n, d.k, d.levels) != (d0.n, d0.k, d0.levels) for d in ds):
        return None
    return ds


def fold_records(deltas: Sequence[CompressedDelta], weights: Sequence[float], delta_params: Sequence[torch.Tensor],
                 theta: Optional[Sequence[torch.Tensor]], v: Optional[Sequence[torch.Tensor]], beta0: float,
                 opt: str = "avg", lr: float = 1.0, beta2: float = 0.0, tau: float = 0.0) -> bool:
    """``δ = β0·δ + Σ_c w_c·decode(record_c)`` in message order, then (``theta``) the server optimiser's step — one
    ``flc_fedopt_fold_records`` pass.  False (nothing launched) when the server tensors are not contiguous fp32 tensors
    of one HIP device holding the records' element count (the caller then takes the dense path)."""
    dps = list(delta_params)
    d0 = deltas[0]
    fast = codec._pyrecs()
    if fast is not None and dps:
        try:  # one C call: every tensor checked in place; TypeError: nothing launched, the checks below decide
            fast([d.record for d in deltas], [float(w) for w in weights], d0.n, d0.k, d0.levels, dps,
                 None if theta is None else list(theta), None if v is None else list(v), float(beta0),
                 _lib.FLC_OPT[opt], float(lr), float(beta2), float(tau))
            return True
        except TypeError:
            pass
    if not dps or not all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype is torch.float32 and t.is_contiguous()
                          for t in dps):
        return False
    dev = dps[0].device
    groups = [dps] + ([list(theta)] if theta is not None else []) + ([list(v)] if v is not None else [])
    for g in groups:
        if len(g) != len(dps) or any(not (t.is_cuda and t.device == dev and t.dtype is torch.float32
                                          and t.is_contiguous() and t.numel() == d.numel()) for t, d in zip(g, dps)):
            return False
    d0 = deltas[0]
    if sum(t.numel() for t in dps) != d0.n:
        return False
    recs = [d.record if d.record.device == dev else d.record.to(dev) for d in deltas]
    m, T = len(recs), len(dps)
    _lib.call("flc_fedopt_fold_records", _ptrs(recs), (ctypes.c_float * m)(*[float(w) for w in weights]), m, d0.n,
              d0.k, d0.levels, _ptrs(dps), _ptrs(groups[1]) if theta is not None else None,
              _ptrs(groups[2]) if v is not None else None, (ctypes.c_int64 * T)(*[t.numel() for t in dps]), T,
              float(beta0), _lib.FLC_OPT[opt], float(lr), float(beta2), float(tau), codec._stream(dev))
    return True


def _compressors_of(node) -> List[Compressor]:
    cs = getattr(node, "compressors", None)
    if cs is None:
        cs = getattr(getattr(node, "config", None), "compressors", None)
    if cs is None:
        return []
    return [cs] if isinstance(cs, Compressor) else list(cs)


class CompressedFedOptClientMixin:
    """Mix in before the reference's ``FedOptClient`` (``class C(CompressedFedOptClientMixin, FedOptClient)``):
    ``communicate`` (_fedopt.py:295-308) sends the delta through the client's compressors (``self.compressors``, or
    ``self.config.compressors``: one :class:`~fl_sim_amd.compressors.Compressor` or a sequence applied in order; none
    sends the plain delta).  The server side is :class:`~fl_sim_amd.aggregation.FedOptUpdateMixin`, which folds a
    round of stacked records in one pass (or any reference server, which reads the message's delta unchanged)."""

    def communicate(self, target) -> None:
        # (the parameters as they are: the codec only reads them, and every converting path detaches first)
        delta = compress_delta(list(self.model.parameters()), self._cached_parameters, _compressors_of(self))
        target._received_messages.append(
            client_message_class()(
                **{
                    "client_id": self.client_id,
                    "delta_parameters": delta,
                    "train_samples": len(self.train_loader.dataset),
                    "metrics": self._metrics,
                }
            )
        )
