"""Where the host time of a configs[0] server update goes (cnn_femmist_tiny: 8 tensors, 10 clients): the FedAvg
update through fedopt_update, codec.model_fold, the torch op with prebuilt lists, and the bare C ABI with prebuilt
pointer tables; each leg enqueued back to back (per-call time = max(host, GPU)), plus the host time alone of the
Python checks.  The kernel itself is ~10 us (rocprof)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import _lib, codec  # noqa: E402
from fl_sim_amd import aggregation as fagg  # noqa: E402

SHAPES = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (256, 1568), (256,), (10, 256), (10,)]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
th = [torch.randn(s, generator=g, device=dev) for s in SHAPES]
dl = [torch.zeros(s, device=dev) for s in SHAPES]
msgs = [{"train_samples": 100 * (i + 1), "delta_parameters": [torch.randn(s, generator=g, device=dev) * 1e-3
                                                              for s in SHAPES]} for i in range(10)]
srcs = [m["delta_parameters"] for m in msgs]
flat = [t for m in srcs for t in m]
w = [0.1] * 10
op = codec._model_fold_op()
P = ctypes.c_void_p
nt = len(SHAPES)
dp = (P * nt)(*[t.data_ptr() for t in dl])
tp = (P * nt)(*[t.data_ptr() for t in th])
sp = (P * len(flat))(*[t.data_ptr() for t in flat])
wt = (ctypes.c_float * 10)(*w)
sz = (ctypes.c_int64 * nt)(*[t.numel() for t in dl])
lib = _lib.load()
st = torch.cuda.current_stream(dev).cuda_stream


def cabi():
    lib.flc_model_fold(ctypes.cast(dp, P), ctypes.cast(sp, P), ctypes.cast(wt, P), 10, ctypes.cast(sz, P), nt, 0, 0.0,
                       ctypes.cast(tp, P), None, 0, 1.0, 0.0, 1e-3, st)


legs = (("fedopt_update", lambda: fagg.fedopt_update(th, dl, None, msgs, "avg", 1.0, (0.0, 1.0), 1e-3)),
        ("codec.model_fold", lambda: codec.model_fold(dl, srcs, w, 0, 0.0, theta=th, opt="avg")),
        ("torch_op_prebuilt", lambda: op(dl, flat, w, 0, 0.0, th, [], 0, 1.0, 0.0, 1e-3)),
        ("c_abi_prebuilt", cabi))
for name, fn in legs:
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: {(t2 - t0) * 1e6 / 200:.2f} us/call, host enqueue {(t1 - t0) * 1e6 / 200:.2f} us/call", flush=True)

# the reference's placement: the server model and its FedOpt state in host memory, the messages on the device
import types  # noqa: E402

from fl_sim_amd.aggregation import FedOptUpdateMixin  # noqa: E402


class HostServer(FedOptUpdateMixin):
    pass


hs = HostServer()
hs.model = torch.nn.Module()
for i, sh in enumerate(SHAPES):
    hs.model.register_parameter(f"p{i}", torch.nn.Parameter(torch.randn(sh)))
hs.delta_parameters = [torch.zeros(sh) for sh in SHAPES]
hs.v_parameters = None
hs.config = types.SimpleNamespace(optimizer="avg", lr=1.0, betas=(0.0, 1.0), tau=1e-3)
hs._received_messages = msgs
for _ in range(10):
    hs.update()
t0 = time.perf_counter()
for _ in range(100):
    hs.update()
print(f"host_server_fedavg: {(time.perf_counter() - t0) * 1e6 / 100:.2f} us/call (host to host, synchronised)", flush=True)
import cProfile  # noqa: E402
import pstats  # noqa: E402

pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    hs.update()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
