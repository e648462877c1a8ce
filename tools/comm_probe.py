"""Host cost of the pieces of one compressed client message (compressed.py: communicate -> compress_delta ->
_stacked_fast), each timed alone over many calls at configs[0]'s model (8 tensors, 417,482 parameters), philox
stacked pipeline.  The GPU work the calls enqueue is drained between pieces, so each figure is host time.
    python tools/comm_probe.py > gpurun_out/<tag>/comm_probe.txt"""
import math
import os
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from fl_sim_amd import Compressor, codec, compressed  # noqa: E402
from fl_sim_amd.compressed import CompressedFedOptClientMixin  # noqa: E402

N = 400


def per_call(fn, n=N):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    return t


def main():
    dev = torch.device("cuda", 0)
    th0 = [torch.randn(s, device=dev) for s in bench.CONFIG0_SHAPES]
    d0 = sum(t.numel() for t in th0)

    class C(CompressedFedOptClientMixin):
        pass

    c = C()
    c.client_id, c._metrics = 0, {}
    c.train_loader = types.SimpleNamespace(dataset=range(100))
    c.model = torch.nn.Module()
    for j, t in enumerate(th0):
        c.model.register_parameter(f"p{j}", torch.nn.Parameter(t + torch.randn_like(t) * 1e-2))
    c._cached_parameters = [t.clone() for t in th0]
    tk = Compressor(rng="philox", seed=0)
    tk.makeTopKCompressor(d0 // 100, d0)
    nc = Compressor("norm")
    nc.makeIdenticalCompressor()
    sd = Compressor(rng="philox", seed=0, extended_levels=True)
    sd.makeStandardDitheringFP32(127, nc, np.inf)
    c.compressors = [tk, sd]
    srv = types.SimpleNamespace(_received_messages=[])

    local = list(c.model.parameters())
    K, s = d0 // 100, 127
    stride, _ = codec.stacked_wire_layout(d0, K)
    fast = codec._pydelta()
    rec = torch.empty(stride, dtype=torch.uint8, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    ws = codec.workspace(dev, codec._ws_size(dev, "flc_stacked_encode_delta_workspace_size", d0, K, len(local)), "topk")
    pieces = {
        "communicate (whole)": lambda: (srv._received_messages.clear(), c.communicate(srv)),
        "compress_delta (whole)": lambda: compressed.compress_delta(local, c._cached_parameters, c.compressors),
        "C call stacked_delta_record": lambda: fast(local, c._cached_parameters, K, s, 1, 2, rec, cnt, ws),
        "list(model.parameters())": lambda: list(c.model.parameters()),
        "shapes + n": lambda: ([t.shape for t in local], sum(t.numel() for t in local)),
        "stacked_pipeline": lambda: compressed.stacked_pipeline(c.compressors),
        "philox.next": lambda: sd.philox.next(),
        "stacked_wire_layout": lambda: codec.stacked_wire_layout(d0, K),
        "torch.empty(record)": lambda: torch.empty(stride, dtype=torch.uint8, device=dev),
        "_count_slot": lambda: sd._count_slot(dev),
        "workspace + _ws_size": lambda: codec.workspace(
            dev, codec._ws_size(dev, "flc_stacked_encode_delta_workspace_size", d0, K, len(local)), "topk"),
        "_stream": lambda: codec._stream(dev),
        "_after_encode": lambda: codec._after_encode(dev),
        "tk._finish": lambda: tk._finish(d0, tk.K),
        "_norm_stage_send": lambda: compressed._norm_stage_send(sd, None),
        "CompressedDelta(...)": lambda: compressed.CompressedDelta([t.shape for t in local], dev, d0, record=rec, k=K,
                                                                   levels=s),
        "client_message_class()(...)": lambda: compressed.client_message_class()(
            client_id=0, delta_parameters=None, train_samples=100, metrics={}),
        "per (log2)": lambda: (1.0 + np.ceil(math.log2(sd.s))) / 32.0,
    }
    only = os.environ.get("ONLY")  # (one piece, e.g. under rocprofv3 --hip-trace --stats)
    for name, fn in pieces.items():
        if only and not name.startswith(only):
            continue
        print(f"{name:34s} {per_call(fn):7.2f} us", flush=True)
        sd.resetStats()  # (the pending counts of the timed calls)


if __name__ == "__main__":
    main()
