"""The aggregation kernels under rocprofv3 --kernel-trace --stats (profiles/r03/*agg*): FedAvg / FedDyn / pFedMe /
FedAdam server updates and avg_parameters at configs[0]'s model x 10 clients, and one weighted fold of 8 x 25 M
(flc_weighted_sum)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fl_sim_amd import aggregation as fagg  # noqa: E402
from fl_sim_amd import codec  # noqa: E402

SHAPES = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (256, 1568), (256,), (10, 256), (10,)]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
th = [torch.randn(s, generator=g, device=dev) for s in SHAPES]
dl = [torch.zeros(s, device=dev) for s in SHAPES]
v = [torch.rand(s, generator=g, device=dev) * 1e-4 + 1e-6 for s in SHAPES]
msgs = [{"train_samples": 100 * (i + 1), "delta_parameters": [torch.randn(s, generator=g, device=dev) * 1e-3
                                                              for s in SHAPES]} for i in range(10)]
srcs = [torch.randn(25_000_000, generator=g, device=dev) for _ in range(8)]
dst = torch.randn(25_000_000, generator=g, device=dev)
w8 = [0.1 * (i + 1) for i in range(8)]
pm = [{"train_samples": m["train_samples"], "parameters": [t + p for t, p in zip(m["delta_parameters"], th)]}
      for m in msgs]
h = [torch.zeros(s, device=dev) for s in SHAPES]
legs = (("fedavg", lambda: fagg.fedopt_update(th, dl, None, msgs, "avg", 1.0, (0.0, 1.0), 1e-3)),
        ("feddyn", lambda: fagg.feddyn_update(th, h, pm, 0.01, 20)),
        ("pfedme", lambda: fagg.pfedme_update(th, pm, 0.7)),
        ("fedadam", lambda: fagg.fedopt_update(th, dl, v, msgs, "adam", 1e-2, (0.9, 0.99), 1e-3)),
        ("avg_parameters", lambda: fagg.avg_parameters(th, msgs, size_aware=True, key="delta_parameters")),
        ("weighted_sum_8x25M", lambda: codec.weighted_sum(dst, srcs, w8, init_mode=0, beta=0.5)))
for name, fn in legs:
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    print(name, "us/call", round((time.perf_counter() - t0) * 1e6 / 50, 2), flush=True)
