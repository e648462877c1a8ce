"""Host-time breakdown of the variance-reduced servers' update on a device-resident model (bench.py vr_update_extra's
shape: configs[0]'s model x 10 clients, vr = True): fused (FedProxUpdateMixin) and two calls, host enqueue against
synchronised time, then cProfile of the fused update (top functions by own time).
    python tools/vr_probe.py > gpurun_out/<tag>/vr_probe.txt"""
import cProfile
import io
import os
import pstats
import sys
import time
import types

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from fl_sim_amd.aggregation import AggregationMixin, FedProxUpdateMixin  # noqa: E402


class Fused(FedProxUpdateMixin):
    pass


class TwoCalls(AggregationMixin):
    def update(self):
        self.avg_parameters()
        if self.config.vr:
            self.update_gradients()


def main():
    dev = torch.device("cuda", 0)
    th0 = [torch.randn(s, device=dev) for s in bench.CONFIG0_SHAPES]
    g = torch.Generator(device=dev).manual_seed(77)
    msgs = [{"client_id": i, "train_samples": 100 * (i + 1),
             "parameters": [t + torch.randn(t.shape, generator=g, device=dev) * 1e-3 for t in th0],
             "gradients": [torch.randn(t.shape, generator=g, device=dev) * 1e-3 for t in th0]} for i in range(10)]
    servers = {}
    for cls in (Fused, TwoCalls):
        s = cls()
        s.model = torch.nn.Module()
        for j, t in enumerate(th0):
            s.model.register_parameter(f"p{j}", torch.nn.Parameter(t.clone()))
        s.config = types.SimpleNamespace(vr=True)
        s._received_messages = msgs
        servers[cls.__name__] = s
    for rep in range(2):
        for name, s in servers.items():
            for _ in range(10):
                s.update()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                s.update()
            host = (time.perf_counter() - t0) / 50
            torch.cuda.synchronize()
            tot = (time.perf_counter() - t0) / 50
            print(f"{name}: host enqueue {host * 1e6:.1f} us, synchronised {tot * 1e6:.1f} us", flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    s = servers["Fused"]
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(50):
        s.update()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"Fused: events around 50 updates {ev[0].elapsed_time(ev[1]) / 50 * 1e3:.1f} us per update")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        s.update()
    torch.cuda.synchronize()
    pr.disable()
    sio = io.StringIO()
    pstats.Stats(pr, stream=sio).sort_stats("tottime").print_stats(25)
    print(sio.getvalue())


if __name__ == "__main__":
    main()
