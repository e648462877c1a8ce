"""Can the fold kernels read and write the server's pinned host tensors in place (zero-copy over PCIe)?  Asks HIP for
the pointer attributes of a torch pinned tensor first (a device kernel must only touch host memory that is mapped
into the device's address space), and only then folds into it with flc_weighted_sum and times it against the
copy-in / fold / copy-out form of fl_sim_amd.hoststage."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import codec  # noqa: E402


class Attr(ctypes.Structure):  # hipPointerAttribute_t (ROCm 6+/7): type, device, devicePointer, hostPointer, ...
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
n = 417_482
h = torch.randn(n).pin_memory()
a = Attr()
rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(h.data_ptr()))
print("rc", rc, "type", a.type, "device", a.device, "host", hex(a.hostPointer or 0), "devptr", hex(a.devicePointer or 0),
      "data_ptr", hex(h.data_ptr()), "flags", a.allocationFlags, flush=True)
if rc != 0 or not a.devicePointer:
    print("not mapped: no zero-copy")
    sys.exit(0)
# fold 10 device messages into the host tensor through the device pointer
msgs = [torch.randn(n, device=dev) * 1e-3 for _ in range(10)]
w = [0.1] * 10
exp = h.clone()
for m in msgs:
    exp.add_(m.cpu(), alpha=0.1)
ptrs = (ctypes.c_void_p * 10)(*[m.data_ptr() for m in msgs])
ws = (ctypes.c_float * 10)(*w)
from fl_sim_amd import _lib  # noqa: E402

st = torch.cuda.current_stream(dev).cuda_stream
_lib.call("flc_weighted_sum", ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(ws, ctypes.c_void_p), 10, n, 2, 0.0,
          ctypes.c_void_p(a.devicePointer), st)
torch.cuda.synchronize()
print("zero-copy fold bit-exact:", torch.equal(h.view(torch.int32), exp.view(torch.int32)), "max diff",
      (h - exp).abs().max().item(), flush=True)
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(50):
        _lib.call("flc_weighted_sum", ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(ws, ctypes.c_void_p), 10, n, 0,
                  0.5, ctypes.c_void_p(a.devicePointer), st)
    torch.cuda.synchronize()
    print(f"zero-copy weighted_sum into host memory: {(time.perf_counter() - t0) * 1e6 / 50:.1f} us/call", flush=True)
d = torch.empty(n, device=dev)
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(50):
        d.copy_(h, non_blocking=True)
        codec.weighted_sum(d, msgs, w, init_mode=0, beta=0.5)
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    print(f"copy in / fold / copy out: {(time.perf_counter() - t0) * 1e6 / 50:.1f} us/call", flush=True)
