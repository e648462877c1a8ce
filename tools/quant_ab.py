"""configs[1]'s one-launch quantizer (flc_quant_encode_auto with the decode fused, 10 x 417,482, 8-bit, p = inf):
per-call wall time over 200 calls and the kernel's own duration (HIP events around each launch, flc_probe), for a
same-box A/B of two prebuilt libraries:  for v in A B A B; do FLC_LIB=ab/libflc_$v.so python tools/quant_ab.py; done"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fl_sim_amd import _lib, codec

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(10, 417_482, generator=g, device=dev) * 1e-3
fn = lambda c: codec.quant_encode_auto(X, 0, 127, seed=0, counter=c)  # noqa: E731
for i in range(50):
    fn(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(200):
    fn(i)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) * 1e6 / 200
_lib.call("flc_probe_set", b"quant_fused_encode_decode")
_lib.call("flc_probe_read", None, None)
for i in range(200):
    fn(i)
torch.cuda.synchronize()
t, c = ctypes.c_double(), ctypes.c_int64()
_lib.call("flc_probe_read", ctypes.byref(t), ctypes.byref(c))
_lib.call("flc_probe_set", None)
print({"lib": os.path.basename(os.environ.get("FLC_LIB", "default")), "us_per_call": round(wall, 2),
       "kernel_us": round(t.value / max(c.value, 1) * 1e3, 2), "launches": c.value,
       "err": codec.quant_status()}, flush=True)
