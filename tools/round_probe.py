"""Host-time breakdown of one configs[0] compressed round (bench.py compressed_round_extra's shape): the round timed
synchronised, then cProfile over 20 rounds (top functions by own time), and the VR update beside it.
    python tools/round_probe.py > gpurun_out/<tag>/round_probe.txt"""

import cProfile
import io
import os
import pstats
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from fl_sim_amd import Compressor  # noqa: E402
from fl_sim_amd.aggregation import FedOptUpdateMixin  # noqa: E402
from fl_sim_amd.compressed import CompressedFedOptClientMixin  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    th0 = [torch.randn(s, device=dev) for s in bench.CONFIG0_SHAPES]
    d0 = sum(t.numel() for t in th0)

    class C(CompressedFedOptClientMixin):
        pass

    class S(FedOptUpdateMixin):
        pass

    clients = []
    for i in range(10):
        c = C()
        c.client_id, c._metrics = i, {}
        c.train_loader = types.SimpleNamespace(dataset=range(100 * (i + 1)))
        c.model = torch.nn.Module()
        for j, t in enumerate(th0):
            c.model.register_parameter(f"p{j}", torch.nn.Parameter(t + torch.randn_like(t) * 1e-2))
        c._cached_parameters = [t.clone() for t in th0]
        tk = Compressor(rng="philox", seed=i)
        tk.makeTopKCompressor(d0 // 100, d0)
        nc = Compressor("norm")
        nc.makeIdenticalCompressor()
        sd = Compressor(rng="philox", seed=i, extended_levels=True)
        sd.makeStandardDitheringFP32(127, nc, np.inf)
        c.compressors = [tk, sd]
        clients.append(c)
    s = S()
    s.model = torch.nn.Module()
    for j, t in enumerate(th0):
        s.model.register_parameter(f"p{j}", torch.nn.Parameter(t.clone()))
    s.delta_parameters = [torch.zeros_like(p) for p in s.model.parameters()]
    s.v_parameters = None
    s.config = types.SimpleNamespace(optimizer="avg", lr=1, betas=(0, 1), tau=1)

    def round_():
        s._received_messages = []
        for c in clients:
            c.communicate(s)
        s.update()

    def comm_only():
        s._received_messages = []
        for c in clients:
            c.communicate(s)

    for fn, name in ((round_, "round"), (comm_only, "10 communicates")):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        host = (time.perf_counter() - t0) / 20
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) / 20
        print(f"{name}: host enqueue {host * 1e6:.1f} us, synchronised {tot * 1e6:.1f} us")
    # the server update alone (its messages made and drained first): host time, and synchronised
    hu, su = [], []
    for i in range(25):
        comm_only()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.update()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i >= 5:
            hu.append(t1 - t0)
            su.append(t2 - t0)
    print(f"server update alone: host {np.median(hu) * 1e6:.1f} us, synchronised {np.median(su) * 1e6:.1f} us")
    # amortised over 64 rounds with every client's send statistics read at the end (the pending counts folded in):
    # the slab slots against one fresh count tensor per call (the torch.cat read-back)
    def rounds64():
        for _ in range(64):
            round_()
        for c in clients:
            c.compressors[1].really_need_to_send_components

    slot = Compressor._count_slot
    for name, fn in (("slab", slot), ("per-call tensors", lambda self, dev, *a: torch.empty(1, dtype=torch.int64,
                                                                                          device=dev)),
                     ("slab", slot)):
        Compressor._count_slot = fn
        rounds64()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            rounds64()
        torch.cuda.synchronize()
        print(f"64 rounds + statistics read, {name}: {(time.perf_counter() - t0) / 192 * 1e6:.1f} us per round")
    Compressor._count_slot = slot
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        round_()
    torch.cuda.synchronize()
    pr.disable()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(30)
    print(sio.getvalue())


if __name__ == "__main__":
    main()
