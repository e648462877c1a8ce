"""RCCL over xGMI through the C ABI (flc_comm_* / flc_rccl_*): the multi-GPU exchange of the aggregation round for
callers that do not use torch.distributed.  One process per GPU; RCCL is loaded by the
library on first use (inside a torch process it is torch's own RCCL).

    uid = comm.unique_id()                      # on one rank; send the bytes to the others out of band
    c = comm.RcclComm(uid, nranks, rank, device)
    c.allgather(send_records, recv_records)     # the packed-wire round (then codec.stacked_fold_wires)
    c.reduce(partial, out, root=0)              # or the dense round
"""

from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def unique_id() -> bytes:
    """A new RCCL unique id (flc_comm_unique_id), to be shared with every rank of the communicator."""
    n = _lib.size("flc_comm_id_bytes")
    buf = ctypes.create_string_buffer(n)
    _lib.call("flc_comm_unique_id", ctypes.cast(buf, ctypes.c_void_p))
    return buf.raw


class RcclComm:
    """One rank of an RCCL communicator (flc_comm_init); collectives run on the current stream of the tensors'
    device, stream-ordered and asynchronous."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: Optional[int] = None):
        if len(uid) != _lib.size("flc_comm_id_bytes"):
            raise ValueError("not an RCCL unique id")
        self._uid = ctypes.create_string_buffer(uid, len(uid))
        h = ctypes.c_void_p()
        _lib.call("flc_comm_init", ctypes.cast(self._uid, ctypes.c_void_p), int(nranks), int(rank),
                  -1 if device is None else int(device), ctypes.byref(h))
        self._h = h

    @property
    def handle(self) -> int:
        return self._h.value or 0

    def size(self):
        n, r = ctypes.c_int(), ctypes.c_int()
        _lib.call("flc_comm_size", self._h, ctypes.byref(n), ctypes.byref(r))
        return n.value, r.value

    @staticmethod
    def _dev(t: torch.Tensor, dtype, name: str):
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.dtype != dtype or not t.is_contiguous():
            raise TypeError(f"{name} must be a contiguous {dtype} HIP tensor")

    def reduce(self, send: torch.Tensor, recv: Optional[torch.Tensor] = None, root: int = 0) -> Optional[torch.Tensor]:
        """fp32 sum of every rank's ``send`` into ``recv`` on rank ``root`` (flc_rccl_reduce)."""
        self._dev(send, torch.float32, "send")
        if recv is not None:
            self._dev(recv, torch.float32, "recv")
            if recv.numel() != send.numel():
                raise ValueError("recv must hold as many elements as send")
        _lib.call("flc_rccl_reduce", send.data_ptr(), None if recv is None else recv.data_ptr(), send.numel(),
                  int(root), self._h, _stream(send))
        return recv

    def allreduce(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        self._dev(send, torch.float32, "send")
        self._dev(recv, torch.float32, "recv")
        if recv.numel() != send.numel():
            raise ValueError("recv must hold as many elements as send")
        _lib.call("flc_rccl_allreduce", send.data_ptr(), recv.data_ptr(), send.numel(), self._h, _stream(send))
        return recv

    def allgather(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        """Every rank's ``send`` bytes into ``recv`` in rank order (flc_rccl_allgather); uint8 tensors."""
        self._dev(send, torch.uint8, "send")
        self._dev(recv, torch.uint8, "recv")
        n, _ = self.size()
        if recv.numel() != n * send.numel():
            raise ValueError(f"recv must hold nranks x {send.numel()} bytes")
        _lib.call("flc_rccl_allgather", send.data_ptr(), recv.data_ptr(), send.numel(), self._h, _stream(send))
        return recv

    def destroy(self) -> None:
        if self._h.value:
            _lib.call("flc_comm_destroy", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
