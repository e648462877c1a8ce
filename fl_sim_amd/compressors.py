"""Drop-in ``Compressor`` with the reference API, running on MI355X kernels.

Mirrors ``fl_sim/compressors/compressors.py`` (class ``Compressor``, lines 35-419; ``CompressorType``,
lines 20-32): the same constructor, ``make*`` factories, properties (``name``/``fullName`` quirks
included), ``getW``, ``resetStats``, send-statistics counters and ``compressVector``/``__call__``
semantics (a new dense decoded vector; the input is never modified).  What changes is where the
work runs: every branch is a gfx950 kernel of ``libflcodec.so`` (see ``codec.py``).

Inputs:
  * ``torch.Tensor`` on a HIP device -> device-resident path, returns a tensor on that device;
  * ``numpy.ndarray`` (or CPU tensor) -> copied to the current HIP device, run there, copied back
    (the reference's own call signature; end-to-end rate incl. PCIe is reported in DESIGN.md).

RNG (``rng=`` constructor argument):
  * ``"compat"`` (default): uniforms come from the interpreter's global ``random`` / ``np.random``
    streams exactly as the reference draws them (one ``random.random()`` per consuming element in
    index order), so outputs are bit-identical to the reference under the same seed;
  * ``"philox"``: counter-based Philox4x32-10 on the device, keyed by ``seed``; no host round trip.

Dithering norm (``norm=`` constructor argument; compressors.py:332, 372 ``np.linalg.norm(x, p)``):
  * ``"auto"`` (default): in compat mode with p != inf, the reference's own norm —
    ``np.float32(np.linalg.norm(x, p))``, the fp32 BLAS dot numpy runs on this host — is computed on the host
    (a device input is copied there for it, as compat mode's uniforms come from the host streams anyway) and
    handed to the kernels, so the output is bit-identical to the reference at any size, for host and device
    inputs alike; otherwise (philox mode, p = inf) the device norm;
  * ``"device"``: always the device norm (p = inf: max |x|, exact; p = 2: an fp64 sum of squares rounded once,
    within 1 ulp of the exact norm, which a float32 BLAS dot is not at large D);
  * ``"reference"``: always the host ``np.linalg.norm`` (a device input is copied to the host for it).

Extensions over the reference (documented in DESIGN.md): ``Compressor(extended_levels=True)`` lets
standard dithering take up to 127 levels (by default level counts > 10 fail the reference's
``np.arange`` assertion, as they do there), ``encode``/``decode`` expose the packed wire, and
``compressBatch`` runs a [clients, d] batch in one launch.
"""

from __future__ import annotations

import math
import random
from enum import Enum, unique
from typing import Any, Optional

import numpy as np
import torch

from . import codec
from . import rng as _rng
from ._lib import FLC_Q_NATURAL_DITHER, FLC_Q_STANDARD_DITHER

__all__ = ["CompressorType", "Compressor"]


@unique
class CompressorType(Enum):
    """Same members and values as the reference enum (compressors.py:20-32)."""

    IDENTICAL = 1
    LAZY_COMPRESSOR = 2
    RANDK_COMPRESSOR = 3
    NATURAL_COMPRESSOR_FP64 = 4
    NATURAL_COMPRESSOR_FP32 = 5
    STANDARD_DITHERING_FP64 = 6
    STANDARD_DITHERING_FP32 = 7
    NATURAL_DITHERING_FP32 = 8
    NATURAL_DITHERING_FP64 = 9
    TOPK_COMPRESSOR = 10
    ADAPTIVE_RANDOM_COMPRESSOR = 11


_BIASED = {CompressorType.TOPK_COMPRESSOR, CompressorType.ADAPTIVE_RANDOM_COMPRESSOR}
_NATURAL = {CompressorType.NATURAL_COMPRESSOR_FP32, CompressorType.NATURAL_COMPRESSOR_FP64}
_STD = {CompressorType.STANDARD_DITHERING_FP32, CompressorType.STANDARD_DITHERING_FP64}
_NATD = {CompressorType.NATURAL_DITHERING_FP32, CompressorType.NATURAL_DITHERING_FP64}


def standard_levels(levels: int) -> np.ndarray:
    """lv[i] = i * (1/s), lv[s] = 1 — bit-equal to the reference's np.arange(0, 1.1, 1/s) (s <= 10)."""
    step = 1.0 / levels
    lv = np.array([i * step for i in range(levels + 1)], dtype=np.float64)
    lv[-1] = 1.0
    return lv


def natural_levels(levels: int) -> np.ndarray:
    """[0, 2^-(s-1), ..., 1/2, 1] (compressors.py:194-197)."""
    lv = np.zeros(levels + 1)
    for i in range(levels):
        lv[i] = (1.0 / 2.0) ** i
    return np.flip(lv)


class Compressor:
    """MI355X-native drop-in for the reference ``Compressor`` (compressors.py:35-419)."""

    def __init__(self, compressorName: str = "", rng: str = "compat", seed: int = 0, extended_levels: bool = False,
                 norm: str = "auto"):
        if rng not in ("compat", "philox"):
            raise ValueError("rng must be 'compat' or 'philox'")
        if norm not in ("auto", "device", "reference"):
            raise ValueError("norm must be 'auto', 'device' or 'reference'")
        self.norm_mode = norm
        # extension: standard dithering with 11..127 levels (8-bit codes); off by default, where such level
        # counts fail the reference's assertion exactly as they do there
        self.extended_levels = bool(extended_levels)
        self.__compressorName = compressorName
        self.__compressorType = CompressorType.IDENTICAL
        self.__w = 0.0
        self._pending = None  # (device count, base, per): send statistics a compressed round left on the device
        self.total_input_components = 0
        self.really_need_to_send_components = 0
        self.last_input_advance = 0
        self.last_need_to_send_advance = 0
        self.rng_mode = rng
        self.philox = _rng.PhiloxStream(seed)

    def __getstate__(self):
        """Copies and pickles carry the folded send statistics: the counts still pending on the device are read back
        (running any deferred encode that writes them) and the per-process device slab is left behind."""
        self._flush()
        d = self.__dict__.copy()
        for key in ("_slab", "_slab_streams"):
            d.pop(key, None)
        return d

    # ------------------------------------------------------------------ properties (compressors.py:58-132)
    @property
    def compressorName(self):
        return self.__compressorName

    @property
    def compressorType(self):
        return self.__compressorType

    @property
    def is_biased(self):
        return self.__compressorType in _BIASED

    @property
    def is_unbiased(self):
        return not self.is_biased

    @property
    def w(self):
        return self.__w

    @property
    def name(self):
        omega = r"$\omega$"
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            return "Identical"
        if t == CompressorType.LAZY_COMPRESSOR:
            return f"Bernoulli(Lazy) [p={self.P:g},{omega}={self.getW():.1f}]"
        if t == CompressorType.RANDK_COMPRESSOR:
            return f"Random-K (K={self.K}) Compressor"
        if t == CompressorType.TOPK_COMPRESSOR:
            return f"Top-K (K={self.K}) Compressor"
        if t == CompressorType.NATURAL_COMPRESSOR_FP64:
            return f"Natural for fp64 [{omega}={self.getW():.1f}]"
        if t == CompressorType.NATURAL_COMPRESSOR_FP32:
            return f"Natural for fp32 [{omega}={self.getW():.1f}]"
        if t == CompressorType.STANDARD_DITHERING_FP64:
            return f"Standard Dithering for fp64[s={self.s}]"
        # the reference tests STANDARD_DITHERING_FP64 twice (compressors.py:93-96), so FP32 falls to "?"
        if t == CompressorType.NATURAL_DITHERING_FP32:
            return f"Natural Dithering for fp32[s={self.s},{omega}={self.getW():.1f}]"
        if t == CompressorType.NATURAL_DITHERING_FP64:
            return f"Natural Dithering for fp64[s={self.s},{omega}={self.getW():.1f}]"
        if t == CompressorType.ADAPTIVE_RANDOM_COMPRESSOR:
            return "Adaptive Random Compressor"
        return "?"

    @property
    def fullName(self):
        omega = r"$\omega$"
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            return "Identical"
        if t == CompressorType.LAZY_COMPRESSOR:
            return f"Bernoulli(Lazy) [p={self.P:g},{omega}={self.getW():.1f}]"
        if t == CompressorType.RANDK_COMPRESSOR:
            return f"Rand [K={self.K},D={self.D}]"
        if t == CompressorType.TOPK_COMPRESSOR:
            return f"Top [K={self.K},D={self.D}]"
        if t == CompressorType.NATURAL_COMPRESSOR_FP64:
            return f"Natural for fp64 [{omega}={self.getW():.1f}]"
        if t == CompressorType.NATURAL_COMPRESSOR_FP32:
            return f"Natural for fp32 [{omega}={self.getW():.1f}]"
        if t == CompressorType.STANDARD_DITHERING_FP64:
            return f"Standard Dithering for fp64[s={self.s}]"
        if t == CompressorType.NATURAL_DITHERING_FP32:
            return f"Natural Dithering for fp32[s={self.s},{omega}={self.getW():.1f}]"
        if t == CompressorType.NATURAL_DITHERING_FP64:
            return f"Natural Dithering for fp64[s={self.s},{omega}={self.getW():.1f}]"
        if t == CompressorType.ADAPTIVE_RANDOM_COMPRESSOR:
            return f"Adaptive Random [D={self.D}]"
        return "?"

    # send statistics (compressors.py:40-43, 406-408).  A compressed client round in philox mode (compressed.py) leaves
    # the dithering stage's count of nonzero inputs on the device instead of synchronising for it; the counts of up to
    # 64 calls wait there and are folded into the counters, in call order with the reference's arithmetic
    # (base + nnz * per per call), the first time one of them is read (one device-to-host copy for all of them).  The
    # counts are written into consecutive slots of one device slab per compressor (_count_slot), so the fold reads
    # them with a single copy of the slab's prefix.
    _kMaxPending = 64

    def _count_slot(self, dev, stream=None) -> torch.Tensor:
        """The one-element int64 device slot for the next pending send count (see _finish_pending); ``stream``: the
        current stream of ``dev`` when the caller has it."""
        pend = self.__dict__.get("_pending") or []
        slab = self.__dict__.get("_slab")
        if len(pend) >= self._kMaxPending or (slab is not None and slab.device != dev):
            self._flush()  # (reads the slab back, so its slots are free again)
            pend = []
        if slab is None or slab.device != dev:
            slab = torch.empty(self._kMaxPending, dtype=torch.int64, device=dev)
            self._slab = slab
        if slab.is_cuda:  # the streams the slots are written on (the read-back waits for each)
            self._note_slab_stream(stream if stream is not None else torch.cuda.current_stream(slab.device))
        return slab[len(pend):len(pend) + 1]

    _before_read = None  # compressed.py: runs the deferred encodes, which write their pending counts

    def _note_slab_stream(self, st) -> None:
        ws = self.__dict__.get("_slab_streams") or []
        if st not in ws:
            self._slab_streams = ws + [st]

    def _flush(self) -> None:
        p = self.__dict__.get("_pending")
        if p and Compressor._before_read is not None:
            Compressor._before_read()
        ws = self.__dict__.get("_slab_streams")
        if ws:
            self._slab_streams = None
            if p:  # counts written on another stream than the one reading them back: order the read after them
                cur = torch.cuda.current_stream(ws[0].device)
                for w in ws:
                    if w != cur:
                        cur.wait_stream(w)
        if p:
            self._pending = None
            cs = [c for c, _, _ in p]
            slab = self.__dict__.get("_slab")
            if slab is not None and all(c.device == slab.device and c.data_ptr() == slab.data_ptr() + 8 * i
                                        for i, c in enumerate(cs)):
                nnzs = [int(v) for v in slab[:len(cs)].tolist()]  # the counts in their slots, in call order
            elif len(cs) > 1 and all(c.device == cs[0].device for c in cs):
                nnzs = [int(v) for v in torch.cat([c.reshape(-1) for c in cs]).tolist()]
            else:
                nnzs = [int(c.item()) for c in cs]
            for (_, base, per), nnz in zip(p, nnzs):
                send = base + nnz * per if nnz else base
                self._last_send = send
                self._really_send += send

    @property
    def last_need_to_send_advance(self):
        self._flush()
        return self._last_send

    @last_need_to_send_advance.setter
    def last_need_to_send_advance(self, v):
        self._flush()
        self._last_send = v

    @property
    def really_need_to_send_components(self):
        self._flush()
        return self._really_send

    @really_need_to_send_components.setter
    def really_need_to_send_components(self, v):
        self._flush()
        self._really_send = v

    def _finish_pending(self, d: int, count, base, per) -> None:
        """_finish with the send count still on the device (see _flush)."""
        pend = self.__dict__.get("_pending") or []
        if len(pend) >= self._kMaxPending:
            self._flush()
            pend = []
        self.last_input_advance = d
        self.total_input_components += d
        pend.append((count, base, per))  # (the advances are added to the totals on flush)
        self._pending = pend

    def resetStats(self):
        if self.__dict__.get("_pending") and Compressor._before_read is not None:
            Compressor._before_read()  # (deferred encodes write their counts before the slots are handed out again)
        self._pending = None
        self.total_input_components = 0
        self.really_need_to_send_components = 0
        self.last_input_advance = 0
        self.last_need_to_send_advance = 0

    # ------------------------------------------------------------------ factories (compressors.py:140-262)
    def _set(self, name: str, ctype: CompressorType, w: float) -> None:
        self.__compressorName = name
        self.__compressorType = ctype
        self.__w = w

    def makeIdenticalCompressor(self):
        self._set("IdenticalCompressor", CompressorType.IDENTICAL, 0.0)
        self.resetStats()

    def makeLazyCompressor(self, P):
        self._set("LazyCompressor", CompressorType.LAZY_COMPRESSOR, 1.0 / P - 1.0)
        self.P = P
        self.resetStats()

    def _make_std(self, name, ctype, levels, vectorNormCompressor, p):
        # compressors.py:154-182: the type and the table change first, then `assert self.s == levels`
        # fails for every level count whose np.arange(0, 1.1, 1/levels) table is not levels + 1 long
        # (all levels > 10), leaving the object half switched, as the reference does
        self.__compressorName = name
        self.__compressorType = ctype
        if self.extended_levels and 1 <= int(levels) <= 127:
            self.levelsValues = standard_levels(int(levels))  # i * (1/s): the arange table where both exist
        else:
            self.levelsValues = np.arange(0.0, 1.1, 1.0 / levels)
        self.s = len(self.levelsValues) - 1
        assert self.s == levels
        self.p = p
        self.vectorNormCompressor = vectorNormCompressor
        self.__w = 0.0
        self.resetStats()

    def makeStandardDitheringFP64(self, levels, vectorNormCompressor, p=np.inf):
        self._make_std("StandardDitheringFP64", CompressorType.STANDARD_DITHERING_FP64, levels, vectorNormCompressor, p)

    def makeStandardDitheringFP32(self, levels, vectorNormCompressor, p=np.inf):
        self._make_std("StandardDitheringFP32", CompressorType.STANDARD_DITHERING_FP32, levels, vectorNormCompressor, p)

    def makeQSGD_FP64(self, levels, dInput):
        norm_compressor = Compressor("norm_compressor")
        norm_compressor.makeIdenticalCompressor()
        self.makeStandardDitheringFP64(levels, norm_compressor, p=2)
        # Lemma 3.1 of arXiv:1610.02132 (compressors.py:188-189)
        self.__w = min(dInput / (levels * levels), dInput**0.5 / levels)

    def _make_natd(self, name, ctype, levels, dInput, p):
        # compressors.py:191-221 (any level count constructs; the device codec takes up to 127)
        self.__compressorName = name
        self.__compressorType = ctype
        self.levelsValues = natural_levels(int(levels))
        self.s = len(self.levelsValues) - 1
        assert self.s == levels
        self.p = p
        r = min(p, 2)
        self.__w = 1.0 / 8.0 + (dInput ** (1.0 / r)) / (2 ** (self.s - 1)) * min(1, (dInput ** (1.0 / r)) / (2 ** (self.s - 1)))
        self.resetStats()

    def makeNaturalDitheringFP64(self, levels, dInput, p=np.inf):
        self._make_natd("NaturalDitheringFP64", CompressorType.NATURAL_DITHERING_FP64, levels, dInput, p)

    def makeNaturalDitheringFP32(self, levels, dInput, p=np.inf):
        self._make_natd("NaturalDitheringFP32", CompressorType.NATURAL_DITHERING_FP32, levels, dInput, p)

    def makeRandKCompressor(self, K, D):
        self._set("RandKCompressor", CompressorType.RANDK_COMPRESSOR, D / K - 1.0)
        self.D = D
        self.K = K
        self.resetStats()

    def makeTopKCompressor(self, K, D):
        self._set("TopKCompressor", CompressorType.TOPK_COMPRESSOR, 0.0)
        self.D = D
        self.K = K
        self.resetStats()

    def makeNaturalCompressorFP64(self):
        self._set("NaturalCompressorFP64", CompressorType.NATURAL_COMPRESSOR_FP64, 1.0 / 8.0)
        self.resetStats()

    def makeNaturalCompressorFP32(self):
        self._set("NaturalCompressorFP32", CompressorType.NATURAL_COMPRESSOR_FP32, 1.0 / 8.0)
        self.resetStats()

    def makeAdaptiveRandomCompressor(self, D):
        self._set("AdaptiveRandomCompressor", CompressorType.ADAPTIVE_RANDOM_COMPRESSOR, 0.0)
        self.D = D
        self.K = 1
        self.resetStats()

    def getW(self):
        return self.w

    # ------------------------------------------------------------------ codec (compressors.py:267-410)
    def compressVector(self, x):
        """Encode + decode ``x`` (1-D); returns the dense decoded vector like the reference."""
        if isinstance(x, torch.Tensor) and x.device.type == "cuda":
            host_norm = None
            if self._wants_host_norm(device_input=True):
                host_norm = self._reference_norm(x.detach().cpu().numpy().reshape(-1))
            return self._compress_device(x, host_norm)
        # host input: the reference's own signature (numpy); H2D -> kernels -> D2H
        is_tensor = isinstance(x, torch.Tensor)
        arr = x.detach().cpu().numpy() if is_tensor else np.asarray(x)
        if arr.dtype != np.float32 and arr.dtype != np.float64:
            raise TypeError(f"the MI355X codec path takes float32 or float64 vectors; got {arr.dtype}")
        host_norm = self._reference_norm(arr.reshape(-1)) if self._wants_host_norm(device_input=False) else None
        dev = torch.device("cuda", torch.cuda.current_device())
        out = self._compress_device(torch.from_numpy(np.ascontiguousarray(arr)).to(dev, non_blocking=False), host_norm)
        out_host = out.cpu()
        return out_host if is_tensor else out_host.numpy().reshape(arr.shape)

    def __call__(self, vec):
        return self.compressVector(vec)

    def __str__(self):
        return self.name

    def __repr__(self):
        return self.fullName

    # ----------------------------------------------------------------------------------------------
    def _wants_host_norm(self, device_input: bool) -> bool:
        if self.compressorType not in _STD and self.compressorType not in _NATD:
            return False
        if self.norm_mode == "reference":
            return True
        # "auto": the reference's norm wherever the output is meant to be the reference's (compat mode), host or
        # device input (round 4: a device input used to take the device norm, 6e-5 away at 25 M elements)
        return self.norm_mode == "auto" and self.rng_mode == "compat" and not math.isinf(self.p)

    def _reference_norm(self, arr: np.ndarray):
        # compressors.py:332 / 372, evaluated as the reference evaluates it (numpy on this host), in x's dtype
        return arr.dtype.type(np.linalg.norm(arr, self.p))

    def _check_bracket(self, norm: float, consumers: int) -> None:
        # a norm of 0 under nonzero elements (a p = 2 norm whose squares underflowed) leaves y = |x| / 0 = inf
        # without a level bracket: the reference's level loop then indexes past its table (compressors.py:346-347)
        # before it draws for that element
        if norm == 0.0 and consumers > 0:
            n = len(self.levelsValues)
            raise IndexError(f"index {n} is out of bounds for axis 0 with size {n}")

    def _uniforms(self, count: int, device) -> torch.Tensor:
        u = _rng.python_random_doubles(count)
        return torch.from_numpy(u).to(device)

    def _finish(self, d: int, send) -> None:
        self.last_input_advance = d
        self.last_need_to_send_advance = send
        self.really_need_to_send_components += self.last_need_to_send_advance
        self.total_input_components += self.last_input_advance

    def _compress_device(self, x: torch.Tensor, host_norm: Optional[np.float32] = None) -> torch.Tensor:
        if x.dim() != 1:
            raise ValueError("compressVector expects a 1-D vector (d = max(x.shape) in the reference)")
        if x.dtype == torch.float64:
            return self._compress_device_f64(x, host_norm)
        d = x.numel()
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            out = codec.copy(x)
            self._finish(d, d)
            return out
        if t == CompressorType.LAZY_COMPRESSOR:
            testp = random.random() if self.rng_mode == "compat" else self._philox_scalar(x.device)
            if testp < self.P:
                out = codec.scale_div(x, float(np.float32(self.P)))
                self._finish(d, d)
            else:
                out = torch.zeros_like(x)
                self._finish(d, 0)
            return out
        if t == CompressorType.RANDK_COMPRESSOR:
            if self.D != d:
                raise ValueError(f"RandK compressor built for D={self.D} applied to a vector of length {d}")
            if self.rng_mode == "compat":  # the reference's own permutation: numpy's legacy stream, on the host
                S = _rng.numpy_shuffle_prefix(self.D, self.K)
                idx = torch.from_numpy(S).to(x.device)
            else:  # device-native: the K largest of D Philox keys (no host round trip)
                seed, ctr = self.philox.next()
                idx = codec.randk_indices(self.D, int(self.K), seed, ctr, x.device)
            out = codec.randk_apply(x, idx, float(np.float32(self.D / self.K)))
            self._finish(d, self.K)
            return out
        if t == CompressorType.TOPK_COMPRESSOR:
            K = int(self.K)
            if K <= 0 or K >= d:
                # np.argsort(out)[:-K] is empty for K == 0 and K >= d: nothing is zeroed
                out = codec.copy(x)
            else:
                idx, val, tiles = codec.topk_encode(x, K, with_tiles=True)
                out = codec.sparse_decode(idx, val, d, tiles=tiles)
            self._finish(d, self.K)
            return out
        if t == CompressorType.ADAPTIVE_RANDOM_COMPRESSOR:
            return self._adaptive(x, d)
        if t in _NATURAL:
            seed, ctr = self.philox.next()
            compat_u = None
            if self.rng_mode == "compat":
                cnt = int(codec.count_consumers(x.reshape(1, -1), None).item())
                compat_u = self._uniforms(cnt, x.device)
            codes, _ = codec.natural_encode(x, seed, ctr, compat_u, want_nnz=False)
            out = codec.natural_decode(codes, d)
            if t == CompressorType.NATURAL_COMPRESSOR_FP64:
                self._finish(d, 12.0 / 64.0 * d)
            else:
                self._finish(d, 9.0 / 32.0 * d)
            return out
        if t in _STD or t in _NATD:
            if not 1 <= self.s <= 127:
                raise ValueError(f"the device dithering codec takes 1..127 levels (8-bit codes); s = {self.s}")
            kind = FLC_Q_STANDARD_DITHER if t in _STD else FLC_Q_NATURAL_DITHER
            x2 = x.reshape(1, d)
            if host_norm is not None:  # the reference's np.linalg.norm (see the module docstring)
                norms = torch.tensor([host_norm], dtype=torch.float32).to(x.device, non_blocking=True)
            else:
                norms = codec.quant_norm(x2, self.p)
            seed, ctr = self.philox.next()
            compat_u = None
            if self.rng_mode == "compat":
                cnt = int(codec.count_consumers(x2, norms).item())
                self._check_bracket(float(norms.item()), cnt)
                compat_u = self._uniforms(cnt, x.device)
            pkt, out = codec.quant_encode_decode(x2, kind, self.s, norms, seed, ctr, compat_u, want_nnz=(t in _STD))
            out = out.reshape(d)
            if t in _STD:
                pnorm = np.float32(norms.item())
                # the norm goes through the norm compressor (compressors.py:334-337)
                self.vectorNormCompressor.compressVector(np.array([pnorm]))
                send = self.vectorNormCompressor.last_need_to_send_advance
                nnz = int(pkt.nnz.item())
                if nnz:
                    per = (1.0 + np.ceil(math.log2(self.s))) / (64.0 if t == CompressorType.STANDARD_DITHERING_FP64 else 32.0)
                    # repeated += of a multiple of 1/64 is exact below 2^46: equals the reference's loop
                    send = send + nnz * per
                self._finish(d, send)
            else:
                den = 64.0 if t == CompressorType.NATURAL_DITHERING_FP64 else 32.0
                self._finish(d, d * (1.0 + np.ceil(math.log2(self.s))) / den)
            return out
        raise ValueError(f"unknown compressor type {t}")

    def _compress_device_f64(self, x: torch.Tensor, host_norm=None) -> torch.Tensor:
        """The float64 forms (f64.hip): the reference keeps every step in float64 when x is float64
        (compressors.py:267-410); same RNG consumption and send statistics as the float32 path."""
        d = x.numel()
        t = self.compressorType
        if t == CompressorType.IDENTICAL:
            out = codec.copy_f64(x)
            self._finish(d, d)
            return out
        if t == CompressorType.LAZY_COMPRESSOR:
            testp = random.random() if self.rng_mode == "compat" else self._philox_scalar(x.device)
            if testp < self.P:
                out = codec.scale_div_f64(x, float(self.P))  # x / P in float64 (compressors.py:279)
                self._finish(d, d)
            else:
                out = torch.zeros_like(x)
                self._finish(d, 0)
            return out
        if t == CompressorType.RANDK_COMPRESSOR:
            if self.D != d:
                raise ValueError(f"RandK compressor built for D={self.D} applied to a vector of length {d}")
            if self.rng_mode == "compat":
                idx = torch.from_numpy(_rng.numpy_shuffle_prefix(self.D, self.K)).to(x.device)
            else:
                seed, ctr = self.philox.next()
                idx = codec.randk_indices(self.D, int(self.K), seed, ctr, x.device)
            out = codec.randk_apply_f64(x, idx, self.D / self.K)  # a Python float times an fp64 element (290)
            self._finish(d, self.K)
            return out
        if t == CompressorType.TOPK_COMPRESSOR:
            K = int(self.K)
            out = codec.copy_f64(x) if K <= 0 or K >= d else codec.topk_dense_f64(x, K)
            self._finish(d, self.K)
            return out
        if t == CompressorType.ADAPTIVE_RANDOM_COMPRESSOR:
            return self._adaptive(x, d)
        if t in _NATURAL:
            seed, ctr = self.philox.next()
            compat_u = None
            if self.rng_mode == "compat":
                compat_u = self._uniforms(int(codec.count_consumers_f64(x, None).item()), x.device)
            _, out = codec.natural_f64(x, seed, ctr, compat_u)
            self._finish(d, (12.0 / 64.0 if t == CompressorType.NATURAL_COMPRESSOR_FP64 else 9.0 / 32.0) * d)
            return out
        if t in _STD or t in _NATD:
            if not 1 <= self.s <= 127:
                raise ValueError(f"the device dithering codec takes 1..127 levels (8-bit codes); s = {self.s}")
            kind = FLC_Q_STANDARD_DITHER if t in _STD else FLC_Q_NATURAL_DITHER
            if host_norm is not None:
                norm = torch.tensor([float(host_norm)], dtype=torch.float64).to(x.device, non_blocking=True)
            else:
                norm = codec.quant_norm_f64(x, self.p)
            seed, ctr = self.philox.next()
            compat_u = None
            if self.rng_mode == "compat":
                cnt = int(codec.count_consumers_f64(x, norm).item())
                self._check_bracket(float(norm.item()), cnt)
                compat_u = self._uniforms(cnt, x.device)
            _, out, nnz = codec.quant_f64(x, kind, self.s, norm, seed, ctr, compat_u, want_nnz=(t in _STD))
            if t in _STD:
                pnorm = np.float64(norm.item())
                self.vectorNormCompressor.compressVector(np.array([pnorm]))  # compressors.py:334-337
                send = self.vectorNormCompressor.last_need_to_send_advance
                nz = int(nnz.item())
                if nz:
                    per = (1.0 + np.ceil(math.log2(self.s))) / (64.0 if t == CompressorType.STANDARD_DITHERING_FP64 else 32.0)
                    send = send + nz * per
                self._finish(d, send)
            else:
                den = 64.0 if t == CompressorType.NATURAL_DITHERING_FP64 else 32.0
                self._finish(d, d * (1.0 + np.ceil(math.log2(self.s))) / den)
            return out
        raise ValueError(f"unknown compressor type {t}")

    def _adaptive(self, x: torch.Tensor, d: int) -> torch.Tensor:
        # np.random.choice(np.arange(self.D), size=1, p=|x| / sum|x|)  (compressors.py:297-301), in x's dtype
        if self.D != d:
            raise ValueError("'a' and 'p' must have same size")
        status = int(codec.adaptive_prepare(x).item())  # numpy checks p before drawing
        if status:
            raise ValueError(codec.ADAPTIVE_ERRORS.get(status, "invalid probabilities"))
        u = _rng.numpy_random_sample() if self.rng_mode == "compat" else self._philox_scalar(x.device)
        out, _ = codec.adaptive_select(x, u)
        self._finish(d, 1)
        return out

    def _philox_scalar(self, device) -> float:
        # one uniform for the Lazy compressor in philox mode (host-side draw from the same key)
        seed, ctr = self.philox.next()
        g = np.random.Generator(np.random.Philox(key=seed, counter=ctr))
        return float(g.random())

    # ------------------------------------------------------------------ extensions
    def compressBatch(self, X: torch.Tensor) -> torch.Tensor:
        """[clients, d] batch of deltas in one launch per kernel (dithering types, philox RNG; top-k: the clients'
        selects in one launch, flc_topk_encode_batch, each row then decoded)."""
        t = self.compressorType
        if t == CompressorType.TOPK_COMPRESSOR:
            X2 = X.reshape(X.shape[0], -1)
            out = torch.empty_like(X2)
            for c, (idx, val, tiles) in enumerate(codec.topk_encode_batch(list(X2.unbind(0)), int(self.K), True)):
                codec.sparse_decode(idx, val, X2.shape[1], out=out[c], tiles=tiles)
            return out.reshape(X.shape)
        if t not in _STD and t not in _NATD:
            raise NotImplementedError("compressBatch: dithering and top-k compressors only")
        kind = FLC_Q_STANDARD_DITHER if t in _STD else FLC_Q_NATURAL_DITHER
        seed, ctr = self.philox.next()
        return codec.quant_encode_auto(X, kind, self.s, self.p, seed, ctr)[1]

    def encode(self, x: torch.Tensor) -> Any:
        """Wire packet of ``x`` (device tensors, philox RNG): QuantPacket / (idx, val, tiles) / StackedPacket."""
        t = self.compressorType
        if t in _STD or t in _NATD:
            kind = FLC_Q_STANDARD_DITHER if t in _STD else FLC_Q_NATURAL_DITHER
            x2 = x.reshape(1, -1)
            seed, ctr = self.philox.next()
            return codec.quant_encode(x2, kind, self.s, codec.quant_norm(x2, self.p), seed, ctr, None, want_nnz=False)
        if t == CompressorType.TOPK_COMPRESSOR:
            return codec.topk_encode(x, int(self.K), with_tiles=True)
        if t in _NATURAL:
            seed, ctr = self.philox.next()
            return codec.natural_encode(x, seed, ctr, None, want_nnz=False)[0]
        raise NotImplementedError(f"encode: {t}")

    def decode(self, packet: Any, d: Optional[int] = None) -> torch.Tensor:
        t = self.compressorType
        if t in _STD or t in _NATD:
            return codec.quant_decode(packet).reshape(-1)
        if t == CompressorType.TOPK_COMPRESSOR:
            idx, val = packet[0], packet[1]
            tiles = packet[2] if len(packet) > 2 else None
            return codec.sparse_decode(idx, val, int(d if d is not None else self.D), tiles=tiles)
        if t in _NATURAL:
            return codec.natural_decode(packet, int(d if d is not None else packet.numel()))
        raise NotImplementedError(f"decode: {t}")
