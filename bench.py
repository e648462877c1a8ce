"""Benchmark of the MI355X gradient-codec path (BASELINE.json metric).

Headline workload (``value``): BASELINE.json configs[4] at one client per GPU — a 1 GiB flat fp32
delta (268,435,456 elements) through the stacked codec: top-k 1 % (k = 2,684,354) then 8-bit
standard dithering (s = 127, p = inf, Philox RNG) of the kept values; one step = encode + decode,
device-resident (input already in HBM when the timed region starts).  GB/s counts the algorithmic
bytes of SURVEY.md §8(d): 8·D + 10·K per client (read x, write dense output, write + read the
5-byte/entry wire).  At N GPUs each rank owns its own client delta (weak scaling), no collective in
the timed region; ``value`` = N x per-client bytes / max-over-ranks step time.

Also reported (``configs``): configs[1] (8-bit dithering of 10 cnn_femmist_tiny deltas batched),
configs[2] (top-k 1 % of a 25M delta), and at N > 1 configs[3] (codec + fused weighted
decode-accumulate + RCCL reduce of a 25M delta per client).  ``roofline`` is the dominant kernel
(stacked_encode: the fused filter + select + compaction kernel) — its algorithmic bytes over its live
HIP-event duration, timed in a separate short run so no event sits inside the timed steps;
``extra.kernels_us`` times every kernel of the step the same way and ``extra.roofline_decode`` gives
the decode kernel's figure.  ``cpu_baseline`` times the CPU-PyTorch path of the same workload on this
host (all threads on the full delta, one thread on a 64 MiB sample) and, labelled apart, the numpy oracle.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--skip-extra] [--skip-cpu]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "grad-codec GB/s (device-resident encode+decode), flat fp32 delta, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GUIDE_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy)
XGMI_GBS = 7 * 153.0  # 7 xGMI links x ~153 GB/s per GPU
D_HEADLINE = 268_435_456
LEVELS = 127


def launch_ranks(n: int, argv) -> int:
    """`--gpus N` without a torch.distributed environment: start N ranks as ONE child launcher.

    This process has not touched the GPU (only `import torch`), and it is never replaced by another
    program: torch.distributed.run runs as a child and its exit status is returned.
    """
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def dist_setup(n_gpus: int, backend: str = "nccl"):
    """Join the process group the launcher made, pin this rank's GPU, and check the world size."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        print(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}; refusing to report a different GPU count",
              file=sys.stderr)
        sys.exit(3)
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":  # RCCL over xGMI
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != n_gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, expected {n_gpus}", file=sys.stderr)
            sys.exit(3)
    elif backend == "nccl":
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(v: float, world: int) -> float:
    if world == 1:
        return v
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def launch_check(world: int, rank: int) -> None:
    """Every rank reports in over the process group; rank 0 prints which ranks it saw."""
    ranks = [rank]
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([rank], dtype=torch.int64)
        got = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(got, t)
        ranks = [int(g.item()) for g in got]
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
    else:
        pids = [os.getpid()]
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks": ranks, "distinct_pids": len(set(pids))}))
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


def settle_gpu(buf: torch.Tensor, seconds: float = 0.2) -> None:
    """Keep the device busy for `seconds` before any warmup step (setup, untimed).  In a fresh process the
    GPU runs steps ~5-18 of the headline 3-5 % slow (406-417 vs 394 us) even after idling 0.2 s, and not at
    all after 0.2 s of sustained memory traffic: a power/clock transition that follows the onset of load
    (tools/coldstart.py, profiles/r02/r02e_coldstart_steps.txt).  The driver's `--warmup 5` would otherwise
    time exactly that transition."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        buf.zero_()
        torch.cuda.synchronize()


def stream_copy_gbs(src: torch.Tensor, dst: torch.Tensor, world: int) -> float:
    """The box's stream-copy rate: 2 * 4 * D bytes per device-to-device copy of src into dst (torch's copy kernel and
    flc_copy, 10 copies each after 3 warm ones; the better of the two), max over ranks of the time."""
    from fl_sim_amd import _lib

    st = lambda: torch.cuda.current_stream(src.device).cuda_stream  # noqa: E731
    best = None
    for fn in (lambda: dst.copy_(src),
               lambda: _lib.call("flc_copy", src.data_ptr(), src.numel(), dst.data_ptr(), st())):
        ms, _ = timed(fn, 10, 3, world)
        ms = max_over_ranks(ms, world)
        best = ms if best is None else min(best, ms)
    return 8 * src.numel() / (best * 1e-3) / 1e9


def stacked_bytes(D: int, K: int) -> int:
    return 8 * D + 10 * K


def timed(fn, steps, warmup, world, probe=None):
    """Barrier+sync bracketed timing of `steps` calls; optional live HIP-event probe of one kernel."""
    from fl_sim_amd import _lib

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if probe:
        _lib.call("flc_probe_set", probe.encode())
        _lib.call("flc_probe_read", None, None)  # clear
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    probe_ms = None
    if probe:
        import ctypes

        tot = ctypes.c_double()
        cnt = ctypes.c_int64()
        _lib.call("flc_probe_read", ctypes.byref(tot), ctypes.byref(cnt))
        _lib.call("flc_probe_set", None)
        probe_ms = tot.value / max(cnt.value, 1)
    return (t1 - t0) * 1e3 / steps, probe_ms


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _time_reps(fn, budget_s: float, max_reps: int, warm: bool = True):
    if warm:
        fn()  # allocator, thread pool
    reps, tot = 0, 0.0
    while reps < max_reps and (reps == 0 or tot < budget_s):
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
        reps += 1
    return tot / reps, reps


def cpu_baseline():
    """north_star's CPU baseline: the CPU-PyTorch path of the same workload (oracle/torch_ref.py: torch.topk, the
    dithering, a dense scatter) on this host's cores, on the full 1 GiB delta at 1 thread, at 16 threads (the box's
    CPU share per GPU) and at all threads; ``value`` is the best of the three, the others are labelled beside it.
    The numpy oracle (oracle/compressors_ref.py, one core) on a 64 MiB sample is a separately labelled field.  Rates
    use the same algorithmic bytes as `value` (8 D + 10 K)."""
    from oracle import compressors_ref as ref
    from oracle import torch_ref

    threads0 = torch.get_num_threads()
    all_threads = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = all_threads
    gen = torch.Generator().manual_seed(1234)
    x_full = torch.randn(D_HEADLINE, generator=gen) * 1e-3
    K = D_HEADLINE // 100
    n_s = 16_777_216  # 64 MiB sample, same K/D ratio
    torch_ref.stacked_step(x_full[:n_s].clone(), n_s // 100, LEVELS, gen)  # warm the pool on a sample
    runs = {}
    for th in sorted({1, min(16, all_threads), all_threads}):
        torch.set_num_threads(th)
        per, reps = _time_reps(lambda: torch_ref.stacked_step(x_full, K, LEVELS, gen), 6.0, 2, warm=False)
        runs[th] = (per, reps)
    torch.set_num_threads(threads0)
    best = min(runs, key=lambda t: runs[t][0])
    per_b, reps_b = runs[best]
    xs = x_full[:n_s].numpy().copy()
    del x_full
    per_np, reps_np = _time_reps(
        lambda: ref.stacked(xs, n_s // 100, LEVELS, lambda i: ref.philox_uniforms_at(i, 1, 0)), 4.0, 3)
    model = cpu_model()
    line = {
        "value": round(stacked_bytes(D_HEADLINE, K) / per_b / 1e9, 4),
        "unit": "GB/s",
        "cores": best,
        "kind": "port",
        "sample": f"CPU-PyTorch stacked top-k 1% -> 8-bit dither (oracle/torch_ref.py: torch.topk + dither + dense "
                  f"scatter) on the full 1 GiB delta; best of 1 / 16 / {all_threads} threads = {best} threads, "
                  f"{reps_b} reps, {per_b * 1e3:.0f} ms/rep; {model}; {affinity} CPUs in this process's affinity mask",
        "cpu_model": model,
        "affinity_cpus": affinity,
        "threads": {str(t): {"value": round(stacked_bytes(D_HEADLINE, K) / runs[t][0] / 1e9, 4), "unit": "GB/s",
                             "ms_per_step": round(runs[t][0] * 1e3, 1), "reps": runs[t][1]} for t in runs},
        "numpy_oracle_1core": {
            "value": round(stacked_bytes(n_s, n_s // 100) / per_np / 1e9, 4), "unit": "GB/s", "cores": 1,
            "sample": f"numpy oracle (oracle/compressors_ref.py stacked, O(n) selection) on a 64 MiB sample, "
                      f"{reps_np} reps, {per_np * 1e3:.0f} ms/rep",
        },
    }
    line["configs"] = cpu_configs(min(16, all_threads))
    return line


CONFIG0_SHAPES = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (256, 1568), (256,), (10, 256), (10,)]  # 417,482


def cpu_configs(threads: int) -> dict:
    """The CPU-PyTorch path beside configs[0]-[3] (BASELINE.md's "cpu_ref, same"), on this host at `threads`
    threads (the box's CPU share per GPU: every op of these small shapes is far slower with all 256 threads of the
    box's cgroup share of 16 cores oversubscribed — 2.6 s for one FedAvg update): configs[0] the reference's FedAvg server update (oracle/aggregation_ref.py: the reference's own torch
    ops) over 10 clients of cnn_femmist_tiny's 8 tensors, configs[1] 8-bit dithering of 10 x 417,482, configs[2]
    top-k 1 % of 25 M with the dense decode, configs[3] 8 clients x 25 M stacked codec + the add_(alpha) fold."""
    from oracle import aggregation_ref, torch_ref

    threads0 = torch.get_num_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(7)
    res = {}
    try:
        theta = [torch.randn(sh, generator=g) for sh in CONFIG0_SHAPES]
        dl = [torch.zeros(sh) for sh in CONFIG0_SHAPES]
        msgs = [{"train_samples": 100 * (i + 1), "delta_parameters": [torch.randn(sh, generator=g) * 1e-3
                                                                      for sh in CONFIG0_SHAPES]} for i in range(10)]
        per, reps = _time_reps(lambda: aggregation_ref.fedopt_update(theta, dl, None, msgs, "avg", 1.0, (0.0, 1.0),
                                                                     1e-3), 1.0, 50)
        res["config0_fedavg_10x417482"] = {"ms": round(per * 1e3, 3), "reps": reps}
        X = torch.randn(10, 417_482, generator=g) * 1e-3
        per, reps = _time_reps(lambda: torch_ref.dither_step(X, LEVELS, g), 2.0, 20)
        res["config1_quant8_10x417482"] = {"ms": round(per * 1e3, 3), "reps": reps,
                                           "GB_s": round(10 * 417_482 * 9 / per / 1e9, 3)}
        x3 = torch.randn(25_000_000, generator=g) * 1e-3
        per, reps = _time_reps(lambda: torch_ref.topk_step(x3, 250_000), 3.0, 5)
        res["config2_topk1pct_25M"] = {"ms": round(per * 1e3, 3), "reps": reps,
                                       "GB_s": round((8 * 25_000_000 + 16 * 250_000) / per / 1e9, 3)}
        w8 = [100 * (i + 1) / 3600 for i in range(8)]
        per, reps = _time_reps(lambda: torch_ref.round_fold([x3] * 8, w8, 250_000, LEVELS, g), 4.0, 2, warm=False)
        res["config3_round_8x25M"] = {"ms": round(per * 1e3, 3), "reps": reps}
        # the codec's call site on the CPU (oracle/round_ref.py: the reference's own composition restated — the client
        # delta, TopK 1 % then standard dithering s = 10 on the host with random.random() uniforms, the FedAvg update)
        from oracle import round_ref

        th = [torch.randn(sh, generator=g) * 0.1 for sh in CONFIG0_SHAPES]
        locs = [[t + torch.randn(t.shape, generator=g) * 1e-2 for t in th] for _ in range(10)]
        dl0 = [torch.zeros(sh) for sh in CONFIG0_SHAPES]
        per, reps = _time_reps(lambda: round_ref.fedopt_round("stacked10", [t.clone() for t in th], dl0, None, locs,
                                                              [100] * 10, "avg", 1.0, (0, 1), 1.0), 2.0, 3)
        res["config0_compressed_round_stacked"] = {"ms": round(per * 1e3, 3), "reps": reps}
    finally:
        torch.set_num_threads(threads0)
    res["threads"] = threads
    return res


def traffic_from_profiles():
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return {}


def compressed_round_extra(dev, world: int, th0) -> dict:
    """The codec at its call site (fl_sim_amd/compressed.py): one configs[0] round — 10 clients (cnn_femmist_tiny on
    the device, nodes.py:706-713) each send their delta (FedOptClient.communicate, _fedopt.py:295-308) through the
    stacked pipeline (TopK 1 %, then standard dithering s = 127, p = inf, of the kept values; philox) as a packed wire
    record; the FedAvg server (FedOptUpdateMixin) folds the records with the server step in one
    flc_fedopt_fold_records pass.  Timed per round: the 10 communicates and the update, the server model on the device
    and in host memory (the reference's placement, nodes.py:606: host to host, synchronised); beside it the same
    round with uncompressed messages (the plain delta, the dense fold)."""
    import types

    from fl_sim_amd import Compressor
    from fl_sim_amd.aggregation import FedOptUpdateMixin
    from fl_sim_amd.compressed import CompressedFedOptClientMixin

    class _Client(CompressedFedOptClientMixin):
        pass

    class _Server(FedOptUpdateMixin):
        pass

    d0, n0 = sum(int(np.prod(s)) for s in CONFIG0_SHAPES), 10
    g = torch.Generator(device=dev).manual_seed(321)
    clients = []
    for i in range(n0):
        c = _Client()
        c.client_id, c._metrics = i, {}
        c.train_loader = types.SimpleNamespace(dataset=range(100 * (i + 1)))
        c.model = torch.nn.Module()
        for j, t in enumerate(th0):
            c.model.register_parameter(f"p{j}", torch.nn.Parameter(t + torch.randn(t.shape, generator=g, device=dev) * 1e-2))
        c._cached_parameters = [t.clone() for t in th0]
        clients.append(c)

    def pipeline(i):
        tk = Compressor(rng="philox", seed=i)
        tk.makeTopKCompressor(d0 // 100, d0)
        nc = Compressor("norm")
        nc.makeIdenticalCompressor()
        sd = Compressor(rng="philox", seed=i, extended_levels=True)
        sd.makeStandardDitheringFP32(LEVELS, nc, np.inf)
        return [tk, sd]

    line = {"model": "cnn_femmist_tiny (8 tensors, 417,482 params) x 10 clients, FedAvg",
            "codec": "TopK 1 % -> standard dithering s = 127 (p = inf) of the kept values, philox"}
    for comp in (True, False):
        for c in clients:
            c.compressors = pipeline(c.client_id) if comp else []
        for where in ("device", "host"):
            s = _Server()
            s.model = torch.nn.Module()
            for j, t in enumerate(th0):
                s.model.register_parameter(f"p{j}", torch.nn.Parameter(t.clone() if where == "device" else t.cpu()))
            s.delta_parameters = [torch.zeros_like(p) for p in s.model.parameters()]
            s.v_parameters = None
            s.config = types.SimpleNamespace(optimizer="avg", lr=1, betas=(0, 1), tau=1)

            def round_():
                s._received_messages = []
                for c in clients:
                    c.communicate(s)
                s.update()

            ms, _ = timed(round_, 20, 5, world)
            key = ("compressed" if comp else "uncompressed") + f"_server_{where}"
            line[key + "_us_per_round"] = round(max_over_ranks(ms, world) * 1e3, 1)
            if comp and where == "device":
                s._received_messages = []
                clients[0].communicate(s)
                line["wire_bytes_per_client"] = s._received_messages[0]["delta_parameters"].nbytes
                line["dense_bytes_per_client"] = 4 * d0
    line["note"] = ("per round: 10 client communicates (delta formed inside the encoder's read, flc_stacked_encode_delta "
                    "into a record) + the server update (flc_fedopt_fold_records: every record decoded and folded in "
                    "message order, the FedAvg step fused); host: the server model adopted into pinned memory and "
                    "updated in place (zero-copy); uncompressed: the plain delta and the dense model fold")
    return line


def vr_update_extra(dev, world: int, th0) -> dict:
    """The variance-reduced servers' update (FedProx, fedprox/_fedprox.py:163-167; FedPD, ProxSkip, pFedMac alike):
    avg_parameters then update_gradients over 10 clients of configs[0]'s model, as one flc_avg_and_gradients launch
    (VRUpdateMixin) against the two calls (AggregationMixin), on the reference's host-resident server and on the
    device.  Algorithmic bytes: 2 n + 2 tensors of 4 D read (parameters, gradients, θ) and 2 written (θ, grads)."""
    import types

    from fl_sim_amd.aggregation import AggregationMixin, FedProxUpdateMixin

    class _Fused(FedProxUpdateMixin):
        pass

    class _TwoCalls(AggregationMixin):
        def update(self):  # fedprox/_fedprox.py:163-167 over the mixin's two methods
            self.avg_parameters()
            if self.config.vr:
                self.update_gradients()

    g = torch.Generator(device=dev).manual_seed(77)
    msgs = [{"client_id": i, "train_samples": 100 * (i + 1),
             "parameters": [t + torch.randn(t.shape, generator=g, device=dev) * 1e-3 for t in th0],
             "gradients": [torch.randn(t.shape, generator=g, device=dev) * 1e-3 for t in th0]} for i in range(10)]
    d0 = sum(t.numel() for t in th0)
    line = {"model": "cnn_femmist_tiny x 10 clients, vr = True",
            "algorithmic_bytes": (2 * 10 + 1) * 4 * d0 + 2 * 4 * d0}
    for cls, name in ((_Fused, "fused"), (_TwoCalls, "two_calls")):
        for where in ("device", "host"):
            s = cls()
            s.model = torch.nn.Module()
            for j, t in enumerate(th0):
                s.model.register_parameter(f"p{j}", torch.nn.Parameter(t.clone() if where == "device" else t.cpu()))
            s.config = types.SimpleNamespace(vr=True)
            s._received_messages = msgs
            ms, _ = timed(s.update, 30, 5, world)
            line[f"{name}_{where}_us"] = round(max_over_ranks(ms, world) * 1e3, 1)
    return line


def aggregation_extras(dev, world: int, rank: int) -> dict:
    """The server half of north_star: the FedAvg and FedAdam server updates
    (FedOptServer.update, _fedopt.py:196-240) and avg_parameters (nodes.py:1134-1163) at configs[0]'s model
    (cnn_femmist_tiny: 8 tensors, 417,482 parameters) x 10 clients — each one flc_model_fold launch for the whole model
    — and one weighted fold of 8 clients x 25 M (flc_weighted_sum, configs[3]'s server fold over dense deltas).
    Algorithmic bytes: a fold reads its n sources and the accumulator and writes it, (n + 2) * 4 * D; the FedOpt
    update additionally reads and writes theta (avg: (n + 4) * 4 * D) and v (adam: (n + 6) * 4 * D)."""
    from fl_sim_amd import aggregation as fagg
    from fl_sim_amd import codec
    from fl_sim_amd import dist as fdist

    out = {}
    ga = torch.Generator(device=dev).manual_seed(99 + rank)
    th0 = [torch.randn(sh, generator=ga, device=dev) for sh in CONFIG0_SHAPES]
    dl0 = [torch.zeros(sh, device=dev) for sh in CONFIG0_SHAPES]
    v0 = [torch.rand(sh, generator=ga, device=dev) * 1e-4 + 1e-6 for sh in CONFIG0_SHAPES]
    msgs0 = [{"train_samples": 100 * (i + 1),
              "delta_parameters": [torch.randn(sh, generator=ga, device=dev) * 1e-3 for sh in CONFIG0_SHAPES]}
             for i in range(10)]
    d0, n0 = 417_482, 10
    legs = {
        "fedavg_update": (lambda: fagg.fedopt_update(th0, dl0, None, msgs0, "avg", 1.0, (0.0, 1.0), 1e-3),
                          (n0 + 4) * 4 * d0),
        "fedadam_update": (lambda: fagg.fedopt_update(th0, dl0, v0, msgs0, "adam", 1e-2, (0.9, 0.99), 1e-3),
                           (n0 + 6) * 4 * d0),
        "avg_parameters": (lambda: fagg.avg_parameters(th0, msgs0, size_aware=True, key="delta_parameters"),
                           (n0 + 2) * 4 * d0),
    }
    line = {"model": "cnn_femmist_tiny (8 tensors, 417,482 params) x 10 clients"}
    for name, (fn, nbytes) in legs.items():
        ms, _ = timed(fn, 50, 10, world)
        ms = max_over_ranks(ms, world)
        gbs = nbytes / (ms * 1e-3) / 1e9
        line[name] = {"us": round(ms * 1e3, 2), "GB_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                      "algorithmic_bytes": nbytes}
    line["bytes_formula"] = ("avg_parameters (n + 2) * 4 * D; FedAvg update (n + 4) * 4 * D, FedAdam (n + 6) * 4 * D; "
                             "D = 417,482, n = 10; the whole model in one flc_model_fold launch (the delta fold and "
                             "the optimizer step fused)")
    out["aggregation_config0_fedavg_10x417482"] = line
    # the reference's own placement (nodes.py:606): the server model and its FedOpt state in HOST memory, the 10
    # clients' messages on the device; FedOptUpdateMixin stages the server's tensors (adopted into one pinned buffer:
    # one H2D and one D2H per update), folds in one launch and writes back in place; host to host, synchronised
    import types

    from fl_sim_amd.aggregation import FedOptUpdateMixin

    class _HostServer(FedOptUpdateMixin):
        pass

    hl = {"model": line["model"], "placement": "server model + delta (+ v) in host memory (nodes.py:606), messages on "
                                               "the device (clients on cuda:i mod N)"}
    for name, opt, lr, betas in (("fedavg_update", "avg", 1.0, (0.0, 1.0)), ("fedadam_update", "adam", 1e-2, (0.9, 0.99))):
        hs = _HostServer()
        hs.model = torch.nn.Module()
        gh = torch.Generator().manual_seed(5)
        for i, sh in enumerate(CONFIG0_SHAPES):
            hs.model.register_parameter(f"p{i}", torch.nn.Parameter(torch.randn(sh, generator=gh)))
        hs.delta_parameters = [torch.zeros(sh) for sh in CONFIG0_SHAPES]
        hs.v_parameters = None if opt == "avg" else [torch.rand(sh, generator=gh) * 1e-4 + 1e-6 for sh in CONFIG0_SHAPES]
        hs.config = types.SimpleNamespace(optimizer=opt, lr=lr, betas=betas, tau=1e-3)
        hs._received_messages = msgs0
        ms_h, _ = timed(hs.update, 50, 10, world)
        ms_h = max_over_ranks(ms_h, world)
        pcie = (2 if opt == "avg" else 3) * 2 * 4 * d0  # theta, delta (, v) each way
        hl[name] = {"us": round(ms_h * 1e3, 2), "pcie_bytes": pcie,
                    "pcie_GB_s": round(pcie / (ms_h * 1e-3) / 1e9, 1)}
    hl["note"] = ("host to host per update: H2D of the server state, one flc_model_fold launch (fold + optimizer step), "
                  "D2H back into the same CPU tensors, stream synchronised; cpu_torch is the reference's CPU update "
                  "with its messages already in host memory")
    out["aggregation_config0_host_server"] = hl
    # FedDyn's and pFedMe's server updates (feddyn/_feddyn.py:172-184, pfedme/_pfedme.py:166-175): one
    # flc_model_fold_server launch each, device-resident, same model and messages (as client parameters)
    pm = [{"train_samples": m["train_samples"], "parameters": [t + p for t, p in zip(m["delta_parameters"], th0)]}
          for m in msgs0]
    h0 = [torch.zeros(sh, device=dev) for sh in CONFIG0_SHAPES]
    srv = {"feddyn_update": (lambda: fagg.feddyn_update(th0, h0, pm, 0.01, 20), (n0 + 4) * 4 * d0),
           "pfedme_update": (lambda: fagg.pfedme_update(th0, pm, 0.7), (n0 + 2) * 4 * d0)}
    sl = {"model": line["model"]}
    for name, (fn, nbytes) in srv.items():
        ms_s, _ = timed(fn, 50, 10, world)
        ms_s = max_over_ranks(ms_s, world)
        sl[name] = {"us": round(ms_s * 1e3, 2), "GB_s": round(nbytes / (ms_s * 1e-3) / 1e9, 1),
                    "algorithmic_bytes": nbytes}
    sl["bytes_formula"] = ("FedDyn (n + 4) * 4 * D: the n messages, theta and h read, theta and h written; pFedMe "
                           "(n + 2) * 4 * D: the n messages and theta read, theta written (the saved model never leaves "
                           "the registers)")
    out["aggregation_config0_feddyn_pfedme"] = sl
    out["compressed_round_config0"] = compressed_round_extra(dev, world, th0)
    out["vr_update_config0"] = vr_update_extra(dev, world, th0)
    del th0, dl0, v0, msgs0
    # 8 x 25 M: distinct sources (a repeated source would be served from the caches)
    n8 = 25_000_000
    srcs8 = [torch.randn(n8, generator=ga, device=dev) * 1e-3 for _ in range(8)]
    dst8 = torch.randn(n8, generator=ga, device=dev) * 1e-3
    w8 = fdist.sample_weights([100 * (i + 1) for i in range(8)])
    fn8 = lambda: codec.weighted_sum(dst8, srcs8, w8, init_mode=0, beta=0.5)  # noqa: E731
    ms8, _ = timed(fn8, 20, 5, world)
    ms8 = max_over_ranks(ms8, world)
    _, kms8 = timed(fn8, 5, 1, world, probe="weighted_sum")
    b8 = (8 + 2) * 4 * n8
    ach = b8 / (kms8 * 1e-3) / 1e9 if kms8 else None
    out["aggregation_weighted_sum_8x25M"] = {
        "ms_per_call": round(ms8, 4), "GB_s": round(b8 / (ms8 * 1e-3) / 1e9, 1),
        "roofline": {"kernel": "weighted_sum", "bound": "hbm", "achieved": None if ach is None else round(ach, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None if ach is None else round(ach / HBM_PEAK_GBS, 4),
                     "avg_us": None if kms8 is None else round(kms8 * 1e3, 1), "algorithmic_bytes": b8},
        "bytes_formula": "(n + 2) * 4 * D: 8 sources + the accumulator read (dst * beta) + dst written",
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)  # the first ~15 steps of a fresh process run ~3 % slow
    ap.add_argument("--skip-extra", action="store_true")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--probe", default="stacked_encode", help="kernel timed live for the roofline entry")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend; gloo only with --launch-check (CPU rehearsal of the launcher)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check the world size, print one JSON line and exit (no GPU work)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.backend != "nccl" and not args.launch_check:
        ap.error("the benchmark itself runs on RCCL; --backend gloo is for --launch-check only")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world, rank, local = dist_setup(args.gpus, args.backend)
    if args.launch_check:
        launch_check(world, rank)
        return
    from fl_sim_amd import codec

    dev = torch.device("cuda", torch.cuda.current_device())
    D, K = D_HEADLINE, D_HEADLINE // 100
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn(D, generator=gen, device=dev) * 1e-3
    out = torch.empty(D, dtype=torch.float32, device=dev)
    settle_gpu(out)
    ctr = [0]

    def step():
        ctr[0] += 1
        pkt = codec.stacked_encode(x, K, LEVELS, seed=rank, counter=ctr[0])
        codec.stacked_decode(pkt, out=out)

    ms, _ = timed(step, args.steps, args.warmup, world)  # no probe events inside the timed steps
    ms = max_over_ranks(ms, world)
    _, probe_ms = timed(step, 5, 1, world, probe=args.probe)  # the roofline kernel, timed on its own run
    value = world * stacked_bytes(D, K) / (ms * 1e-3) / 1e9

    # dominant-kernel roofline: algorithmic bytes per launch / live average duration
    # stacked_encode (sample select + filter + exact select + ordered compaction, one kernel): reads x,
    # writes the wire (idx + code) and the tile pointers; stacked_decode: writes the dense output, reads
    # the wire and the tile pointers
    tiles_b = 4 * (-(-D // 1024) + 1)
    kernel_bytes = {"stacked_encode": 4 * D + 5 * K + tiles_b, "stacked_decode": 4 * D + 5 * K + tiles_b,
                    "topk_filter": 4 * D}
    roof = None
    if probe_ms:
        ach = kernel_bytes.get(args.probe, 4 * D) / (probe_ms * 1e-3) / 1e9
        tr = (traffic_from_profiles().get(args.probe) or {}).get("bytes")
        roof = {
            "kernel": args.probe,
            "bound": "hbm",
            "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": tr,
            "avg_ms": round(probe_ms, 5),
            "algorithmic_bytes": kernel_bytes.get(args.probe),
        }
    if roof is not None:
        # the box's own achievable HBM rate beside the spec peak: a 1 GiB device-to-device copy (read
        # 4 D + write 4 D), the best of torch's copy kernel and flc_copy, timed over its own short run
        cp = stream_copy_gbs(x, out, world)
        roof["stream_copy_GB_s"] = round(cp, 1)
        roof["frac_of_stream_copy"] = round(roof["achieved"] / cp, 4)
        roof["value_frac_of_stream_copy"] = round(value / world / cp, 4)
        # the guide's measured float4 copy (MI355X_MICROARCH.md: 6.29 TB/s), beside the box's own copy: the best copy
        # shape found here (tools/copyprobe.hip, profiles/r05/r05b_copyprobe.txt) reaches 5.9 TB/s, below the codec's
        # own decode write stream, so this copy is a reference point, not a ceiling
        roof["guide_copy_GB_s"] = GUIDE_COPY_GBS
        roof["value_frac_of_guide_copy"] = round(value / world / GUIDE_COPY_GBS, 4)
    extra = {}
    parity = None  # set by the configs[3] legs (skipped with --skip-extra)
    if probe_ms:
        # every kernel of the step, each timed live (HIP events on its launch stream) over its own short run
        kernels = {}
        for name in ("topk_sample", "stacked_encode", "stacked_decode"):
            _, kms = timed(step, 5, 1, world, probe=name)
            if kms:
                kernels[name] = round(kms * 1e3, 1)
        extra["kernels_us"] = kernels
        if kernels.get("stacked_decode"):
            dms = kernels["stacked_decode"] * 1e-3
            ach_d = kernel_bytes["stacked_decode"] / (dms * 1e-3) / 1e9
            extra["roofline_decode"] = {
                "kernel": "stacked_decode", "bound": "hbm", "achieved": round(ach_d, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach_d / HBM_PEAK_GBS, 4),
                "traffic": (traffic_from_profiles().get("stacked_decode") or {}).get("bytes"),
                "algorithmic_bytes": kernel_bytes["stacked_decode"],
            }
    if not args.skip_extra:
        # SURVEY §8(d)'s "realistic" variant of the headline input: 5 % exact zeros (the dithering's zero path,
        # zeros among the candidates); same step, same bytes formula
        xz = x.clone()
        xz[torch.rand(D, generator=gen, device=dev) < 0.05] = 0.0
        cz = [0]

        def step_z():
            cz[0] += 1
            pkt = codec.stacked_encode(xz, K, LEVELS, seed=rank, counter=cz[0])
            codec.stacked_decode(pkt, out=out)

        msz, _ = timed(step_z, args.steps, args.warmup, world)
        msz = max_over_ranks(msz, world)
        extra["headline_5pct_zeros"] = {"ms_per_step": round(msz, 5),
                                        "GB_s": round(world * stacked_bytes(D, K) / (msz * 1e-3) / 1e9, 1)}
        del xz
        # host-resident path (north_star: client state lives on the CPU simulator): pinned host delta ->
        # H2D -> encode + decode -> D2H of the dense decoded vector; PCIe-bound, never `value`
        hx = torch.empty(D, dtype=torch.float32, pin_memory=True)
        hx.copy_(x, non_blocking=False)
        hout = torch.empty(D, dtype=torch.float32, pin_memory=True)
        ce = [0]

        def step_host():
            ce[0] += 1
            x.copy_(hx, non_blocking=True)
            pkt = codec.stacked_encode(x, K, LEVELS, seed=rank, counter=ce[0])
            codec.stacked_decode(pkt, out=out)
            hout.copy_(out, non_blocking=True)

        ms_h, _ = timed(step_host, 3, 1, world)
        ms_h = max_over_ranks(ms_h, world)
        t0 = time.perf_counter()
        for _ in range(3):
            x.copy_(hx, non_blocking=True)
        torch.cuda.synchronize()
        h2d = 3 * 4 * D / (time.perf_counter() - t0) / 1e9
        t0 = time.perf_counter()
        for _ in range(3):
            hout.copy_(out, non_blocking=True)
        torch.cuda.synchronize()
        d2h = 3 * 4 * D / (time.perf_counter() - t0) / 1e9
        extra["e2e_host_sequential"] = {
            "ms_per_step": round(ms_h, 4),
            "GB_s": round(world * stacked_bytes(D, K) / (ms_h * 1e-3) / 1e9, 1),
            "h2d_GB_s": round(h2d, 1),
            "d2h_GB_s": round(d2h, 1),
            "note": "pinned host x -> H2D -> stacked encode+decode -> D2H of the dense output; same bytes formula",
        }
        # the same per client through HostCodecPipeline (f3): client i+1's H2D, client i's codec and client
        # i-1's D2H overlap (6 clients; one pinned input reused, two pinned outputs alternating)
        from fl_sim_amd.host import HostCodecPipeline

        pipe = HostCodecPipeline(D, dev)
        hout2 = torch.empty(D, dtype=torch.float32, pin_memory=True)
        m_cl = 6
        pipe.run([hx] * 2, [hout, hout2], K, LEVELS, seeds=[rank] * 2)  # warm (streams, workspace)
        pipe.synchronize()
        barrier(world)
        t0 = time.perf_counter()
        pipe.run([hx] * m_cl, [hout, hout2] * (m_cl // 2), K, LEVELS, seeds=[rank] * m_cl)
        pipe.synchronize()
        barrier(world)
        ms_p = max_over_ranks((time.perf_counter() - t0) * 1e3 / m_cl, world)
        extra["e2e_host"] = {
            "ms_per_client": round(ms_p, 4),
            "GB_s": round(world * stacked_bytes(D, K) / (ms_p * 1e-3) / 1e9, 1),
            "clients": m_cl,
            "note": "pinned host deltas -> H2D / codec / D2H pipelined across clients (fl_sim_amd.host); "
                    "fill and drain included; same bytes formula",
        }
        # f3 with the packed wire: clients send only their wire to the host (D2H ~14.5 MB per 1 GiB client), the
        # server copies each wire back (H2D) and decodes it into ONE device accumulator with the client's weight
        # fused; one D2H of the aggregate per round.  PCIe carries 4 D + 2 x wire per client instead of 8 D.
        from fl_sim_amd.host import HostWirePipeline

        wp = HostWirePipeline(D, K, LEVELS, dev)
        wires = wp.new_wires(m_cl)
        acc = torch.empty(D, dtype=torch.float32, device=dev)
        wts = [1.0 / m_cl] * m_cl
        wp.encode([hx] * 2, wires[:2], seeds=[rank] * 2)  # warm (streams, workspace, pinned pages)
        wp.decode_accumulate(wires[:2], wts[:2], acc)
        wp.synchronize()
        barrier(world)
        t0 = time.perf_counter()
        wp.encode([hx] * m_cl, wires, seeds=[rank] * m_cl, counters=list(range(m_cl)))
        wp.decode_accumulate(wires, wts, acc)
        wp.wait()
        hout.copy_(acc, non_blocking=True)
        torch.cuda.synchronize()
        barrier(world)
        ms_w = max_over_ranks((time.perf_counter() - t0) * 1e3 / m_cl, world)
        extra["e2e_host_wire"] = {
            "ms_per_client": round(ms_w, 4),
            "GB_s": round(world * stacked_bytes(D, K) / (ms_w * 1e-3) / 1e9, 1),
            "clients": m_cl,
            "wire_bytes_per_client": wires[0].nbytes,
            "note": "pinned host deltas -> H2D -> encode -> D2H of the wire only; server: H2D of each wire -> "
                    "weighted decode-accumulate into one device accumulator -> one D2H of the aggregate "
                    "(fl_sim_amd.host.HostWirePipeline); same bytes formula",
        }
        del hx, hout, hout2, pipe, wp, wires, acc
    del x, out
    torch.cuda.empty_cache()

    if not args.skip_extra:
        # configs[1]: 8-bit dithering, 10 clients x cnn_femmist_tiny (417,482 params), one batched launch
        d2, b2 = 417_482, 10
        X = torch.randn(b2, d2, generator=gen, device=dev) * 1e-3
        c2 = [0]

        def step2():
            c2[0] += 1
            norms = codec.quant_norm(X)
            pkt = codec.quant_encode(X, 0, LEVELS, norms, seed=rank, counter=c2[0], want_nnz=False)
            codec.quant_decode(pkt)

        ms2, _ = timed(step2, 50, 10, world)
        ms2 = max_over_ranks(ms2, world)
        def step2f():  # the same round trip in two launches: norm partials, then encode (norm folded in) + decode
            c2[0] += 1
            codec.quant_encode_auto(X, 0, LEVELS, seed=rank, counter=c2[0])

        ms2f, _ = timed(step2f, 50, 10, world)
        ms2f = max_over_ranks(ms2f, world)
        extra["config2_quant8_10x417482"] = {
            "us_per_step": round(ms2 * 1e3, 2),
            "GB_s": round(b2 * d2 * 10 / (ms2 * 1e-3) / 1e9, 1),
            "bytes_formula": "(8 + 8/4) * D per client (norm, encode, decode reading the wire: 3 launches)",
            "fused_us_per_step": round(ms2f * 1e3, 2),
            "fused_GB_s": round(b2 * d2 * 9 / (ms2f * 1e-3) / 1e9, 1),
            "fused_bytes_formula": "(4 + 1 + 4) * D per client (flc_quant_encode_auto: ONE persistent launch - x read "
                                   "into registers, a grid exchange of the per-row maxima, the codes and the decoded "
                                   "values written from the registers; the wire is not read back)",
        }
        del X
        from fl_sim_amd import dist as fdist

        # configs[2]: top-k 1% of a 25M delta (encode + dense decode).  Fresh inputs: the steps rotate over the 8
        # distinct client deltas of configs[3] (800 MB, above the 256 MiB Infinity Cache), as fl-sim's clients each
        # bring a new delta; the same-input figure (x cache-resident after the first step) is kept beside it
        d3 = 25_000_000
        k3 = d3 // 100
        n_cl4 = 8
        X8 = [fdist.synthetic_client_delta(c, d3, dev) for c in range(n_cl4)]
        X3 = X8[0]
        o3 = torch.empty(d3, dtype=torch.float32, device=dev)
        r3 = [0]

        def step3(rotate=True):  # the TopK compressor's path: encoder-emitted tile pointers, no index pass
            r3[0] += 1
            xi = X8[r3[0] % n_cl4] if rotate else X3
            idx, val, tiles = codec.topk_encode(xi, k3, with_tiles=True)
            codec.sparse_decode(idx, val, d3, out=o3, tiles=tiles)

        ms3, _ = timed(step3, 24, 8, world)
        ms3 = max_over_ranks(ms3, world)
        ms3c, _ = timed(lambda: step3(False), 20, 5, world)
        ms3c = max_over_ranks(ms3c, world)
        extra["config3_topk1pct_25M"] = {
            "ms_per_step": round(ms3, 4),
            "GB_s": round((8 * d3 + 16 * k3) / (ms3 * 1e-3) / 1e9, 1),
            "bytes_formula": "8 * D + 16 * K",
            "inputs": f"{n_cl4} distinct 100 MB deltas in rotation (fresh: not cache-resident)",
            "same_input_ms_per_step": round(ms3c, 4),
        }
        del o3
        # a7: adaptive random (np.random.choice with p = |x| / sum|x|) on a 25M delta, device u (philox mode);
        # rotating over the distinct deltas as above
        ra = [0]

        def step_ar(rotate=True):
            ra[0] += 1
            xi = X8[ra[0] % n_cl4] if rotate else X3
            codec.adaptive_prepare(xi)
            codec.adaptive_select(xi, 0.37)

        ms_ar, _ = timed(step_ar, 16, 8, world)
        ms_ar = max_over_ranks(ms_ar, world)
        ms_arc, _ = timed(lambda: step_ar(False), 10, 3, world)
        ms_arc = max_over_ranks(ms_arc, world)
        extra["adaptive_random_25M"] = {
            "ms_per_call": round(ms_ar, 4),
            "GB_s": round(12 * d3 / (ms_ar * 1e-3) / 1e9, 1),
            "bytes_formula": "12 * D: two reads of x (the buffer sums, the speculated cumsum) + the dense output",
            "inputs": f"{n_cl4} distinct 100 MB deltas in rotation",
            "same_input_ms_per_call": round(ms_arc, 4),
            "note": "bit-exact numpy order: pairwise fp32 sum per 8192-element buffer, speculated exact fp64 cumsum "
                    "(DESIGN.md 3.5); the numpy reference takes ~0.3 s for this call",
        }
        # f1: client delta formation + flatten (FedOptClient.communicate), 1 GiB of parameters in 64 tensors
        sizes5 = [(1 << 22) + (i % 3) for i in range(63)]
        sizes5.append((1 << 28) - sum(sizes5))
        L5 = [torch.randn(n, generator=gen, device=dev) for n in sizes5]
        G5 = [torch.randn(n, generator=gen, device=dev) for n in sizes5]
        o5 = torch.empty(1 << 28, dtype=torch.float32, device=dev)
        ms5, _ = timed(lambda: codec.delta_flatten(L5, G5, out=o5), 20, 5, world)
        ms5 = max_over_ranks(ms5, world)
        extra["f1_client_delta_flatten_1GiB_64_tensors"] = {
            "ms_per_step": round(ms5, 4),
            "GB_s": round(12 * (1 << 28) / (ms5 * 1e-3) / 1e9, 1),
            "bytes_formula": "12 * D (8 read + 4 written)",
        }
        # f1, second half: the client step = delta formation + stacked encode; two passes (delta_flatten writes the
        # flat delta, the encode reads it) against the delta formed inside the encoder's read (stacked_encode_delta)
        k5 = (1 << 28) // 100
        c5 = [0]

        def step5_two():
            c5[0] += 1
            codec.stacked_encode(codec.delta_flatten(L5, G5, out=o5), k5, LEVELS, seed=rank, counter=c5[0])

        def step5_fused():
            c5[0] += 1
            codec.stacked_encode_delta(L5, G5, k5, LEVELS, seed=rank, counter=c5[0])

        ms5t, _ = timed(step5_two, 10, 3, world)
        ms5f, _ = timed(step5_fused, 10, 3, world)
        ms5t, ms5f = max_over_ranks(ms5t, world), max_over_ranks(ms5f, world)
        extra["f1_client_step_delta_plus_encode_1GiB_64_tensors"] = {
            "two_pass_ms": round(ms5t, 4),
            "fused_ms": round(ms5f, 4),
            "fused_GB_s": round((8 * (1 << 28) + 5 * k5) / (ms5f * 1e-3) / 1e9, 1),
            "bytes_formula": "8 * D read (local + global) + 5 * K wire written",
            "plain_encode_us": (extra.get("kernels_us") or {}).get("stacked_encode"),
        }
        del L5, G5, o5
        # a round's many small clients on one GPU (fl-sim's usual case): the stacked encode of 100 clients x 1 M and
        # the delta-fused encode of 10 clients x cnn_femmist-sized tensors, one batched launch against one per client
        gb = torch.Generator(device=dev).manual_seed(77 + rank)
        xs_b = [torch.randn(1_000_000, generator=gb, device=dev) * 1e-3 for _ in range(100)]
        kb = 10_000
        # (30 calls: the first call's ~0.1 ms of host work before its first launch is not amortised over 10)
        msb, _ = timed(lambda: codec.stacked_encode_batch(xs_b, kb, LEVELS, seeds=list(range(100)), counter=1),
                       30, 5, world)
        msb1, _ = timed(lambda: [codec.stacked_encode(x, kb, LEVELS, seed=i, counter=1) for i, x in enumerate(xs_b)],
                        5, 1, world)
        shp = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (2048, 123), (123,), (62, 2048), (62,)]
        glb = [torch.randn(*s, generator=gb, device=dev) for s in shp]
        lcs = [[t + torch.randn(*t.shape, generator=gb, device=dev) * 1e-3 for t in glb] for _ in range(10)]
        nd = sum(t.numel() for t in glb)
        msd, _ = timed(lambda: codec.stacked_encode_delta_batch(lcs, glb, nd // 100, LEVELS, seeds=list(range(10)),
                                                                counter=1), 10, 3, world)
        msd1, _ = timed(lambda: [codec.stacked_encode_delta(lp, glb, nd // 100, LEVELS, seed=i, counter=1)
                                 for i, lp in enumerate(lcs)], 10, 3, world)
        extra["batched_round_encodes"] = {
            "stacked_100x1M_ms": round(max_over_ranks(msb, world), 4),
            "stacked_100x1M_one_launch_per_client_ms": round(max_over_ranks(msb1, world), 4),
            "delta_10x%d_ms" % nd: round(max_over_ranks(msd, world), 4),
            "delta_10x%d_one_launch_per_client_ms" % nd: round(max_over_ranks(msd1, world), 4),
            "note": "flc_stacked_encode_batch / flc_stacked_encode_delta_batch: every client's select on its share of "
                    "the CUs in one launch, packets bit-identical to the per-client encodes (DESIGN.md 3.1b)",
        }
        del xs_b, glb, lcs
        torch.cuda.empty_cache()

        # configs[3]: 8 clients, client i on rank i mod N (nodes.py:706-713), w_i = ts_i / sum ts with
        # ts_i = 100 (i + 1); each rank folds its clients (stacked codec + fused weighted decode-accumulate), then
        # ONE RCCL reduce to rank 0 (none at N = 1: the fold is the whole round).  8 clients at every N: the total
        # work is fixed (strong scaling for this line; the headline is weak scaling).
        acc = torch.empty(d3, dtype=torch.float32, device=dev)
        w_all = fdist.sample_weights([100 * (i + 1) for i in range(n_cl4)])
        mine = fdist.client_shard(n_cl4, world, rank)
        c4 = [0]

        def step4():
            c4[0] += 1
            fdist.aggregate_round([X8[c] for c in mine], [w_all[c] for c in mine], mine,
                                  fdist.stacked_decode_accumulate(k3, LEVELS, seed=0, counter=c4[0]),
                                  out=acc, dst=0)

        ms4, _ = timed(step4, 10, 3, world)
        ms4 = max_over_ranks(ms4, world)

        # the two halves on their own (per-GPU codec rate and reduce time separately):
        # the local fold (encode + weighted decode-accumulate of this rank's clients), then the reduce
        fold = fdist.stacked_decode_accumulate(k3, LEVELS, seed=0, counter=0)

        def step4_codec():  # as aggregate_round does it: the rank's clients into records, one fold from +0
            fold.many([X8[c] for c in mine], [w_all[c] for c in mine], acc, mine, accumulate=False)

        ms4c, _ = timed(step4_codec, 10, 3, world)
        ms4c = max_over_ranks(ms4c, world)
        tiles3 = 4 * (-(-d3 // 1024) + 1)
        # per client: the encode reads x and writes its record (5 K + tiles), the fold reads the record; the fold
        # writes the partial sum once
        codec_b = len(mine) * (4 * d3 + 2 * (5 * k3 + tiles3)) + 4 * d3
        line4 = {
            "ms_per_step": round(ms4, 4),
            "clients": n_cl4,
            "clients_per_rank": len(mine),
            "codec_ms": round(ms4c, 4),
            "codec_GB_s_per_gpu": round(codec_b / (ms4c * 1e-3) / 1e9, 1),
            "codec_GB_s_aggregate": round(world * codec_b / (ms4c * 1e-3) / 1e9, 1),
            "bytes_formula": "codec: n_local * (4 * D + 2 * (5 * K + tiles)) + 4 * D (encode into records, one fold "
                             "from +0 over them); reduce: 4 * D (algBw = busBw)",
        }
        if world > 1:
            import torch.distributed as tdist

            ms4r, _ = timed(lambda: tdist.reduce(acc, dst=0, op=tdist.ReduceOp.SUM), 10, 3, world)
            ms4r = max_over_ranks(ms4r, world)
            line4["reduce_ms"] = round(ms4r, 4)
            # nccl-tests convention for reduce: busBw = algBw = bytes / time (every non-root rank's whole 4 D
            # buffer crosses a link); the timed reduces re-reduce `acc` in place (values unused)
            line4["reduce_algbw_GB_s"] = round(4 * d3 / (ms4r * 1e-3) / 1e9, 1)
            # against the xGMI bound (7 links x ~153 GB/s per GPU)
            line4["reduce_frac_of_xgmi"] = round(4 * d3 / (ms4r * 1e-3) / 1e9 / XGMI_GBS, 4)
        # the same round with the packed wire as the only exchange (SURVEY §8(e)'s sparse alternative): each rank
        # encodes its clients into wire records, ONE all_gather of the records, the fold of all 8 clients in
        # client order in one pass on rank 0 (bit-identical to the single-device fold at every N)
        wc4 = fdist.StackedWireCodec(d3, k3, LEVELS, seed=0, counter=0)

        def step4w():
            c4[0] += 1
            wc4.counter = c4[0]
            fdist.aggregate_round_wire([X8[c] for c in mine], w_all, n_cl4, wc4, out=acc, dst=0, device=dev)

        ms4w, _ = timed(step4w, 10, 3, world)
        ms4w = max_over_ranks(ms4w, world)
        per4 = -(-n_cl4 // world)
        line4["wire_ms_per_step"] = round(ms4w, 4)
        if len(mine) > 1:
            # the same round with one encode launch per client instead of the rank's clients in one batched launch
            # (flc_stacked_encode_batch: each client's select on its share of the CUs)
            class _OneByOne:
                stride, n = wc4.stride, wc4.n
                encode_into, fold = wc4.encode_into, wc4.fold

            def step4w1():
                c4[0] += 1
                wc4.counter = c4[0]
                fdist.aggregate_round_wire([X8[c] for c in mine], w_all, n_cl4, _OneByOne, out=acc, dst=0, device=dev)

            ms4w1, _ = timed(step4w1, 10, 3, world)
            line4["wire_ms_per_step_one_launch_per_client"] = round(max_over_ranks(ms4w1, world), 4)
        if world > 1:
            # the wire exchange alone: one all_gather of every rank's block of records (nccl-tests convention:
            # algBw = world * block / t, busBw = algBw * (world - 1) / world), against the xGMI bound
            import torch.distributed as tdist

            blk = torch.zeros(per4 * wc4.stride, dtype=torch.uint8, device=dev)
            gat = torch.empty(world * blk.numel(), dtype=torch.uint8, device=dev)
            msg, _ = timed(lambda: tdist.all_gather_into_tensor(gat, blk), 10, 3, world)
            msg = max_over_ranks(msg, world)
            alg = world * blk.numel() / (msg * 1e-3) / 1e9
            line4["wire_allgather_ms"] = round(msg, 4)
            line4["wire_allgather_algbw_GB_s"] = round(alg, 1)
            line4["wire_allgather_busbw_GB_s"] = round(alg * (world - 1) / world, 1)
            line4["wire_allgather_frac_of_xgmi"] = round(alg * (world - 1) / world / XGMI_GBS, 4)
            del blk, gat
        line4["xgmi_GB_s"] = XGMI_GBS
        line4["inputs"] = f"{n_cl4} distinct client deltas (dist.synthetic_client_delta), 100 MB each"
        line4["wire_record_bytes"] = wc4.stride
        line4["wire_gather_bytes_per_rank"] = per4 * wc4.stride
        line4["wire_bytes_formula"] = ("codec: n_local * (4 * D + 5 * K + tiles) written as records; all_gather: "
                                       "world * ceil(8 / world) records; fold: 4 * D written + 8 records read")
        extra["config4_codec_plus_rccl_reduce_25M"] = line4
        # self-check: one more round both ways over the process group, compared on rank 0 with the
        # single-device per-client chain of all 8 clients — the wire round bit for bit, the dense round within
        # 1e-6 * sum|w d| + 1e-30
        parity = fdist.round_parity(X8, w_all, fdist.StackedWireCodec(d3, k3, LEVELS, seed=0, counter=777),
                                    fdist.stacked_decode_accumulate(k3, LEVELS, seed=0, counter=777), dst=0,
                                    device=dev)
        del acc
        del X3, X8
        torch.cuda.empty_cache()
        extra.update(aggregation_extras(dev, world, rank))

    # the top-k encoders' sticky error word on every rank (co-residency / count checks, include/flcodec.h), OR-ed
    topk_err = 0
    for v in codec.topk_status_all(reset=True).values():
        topk_err |= int(v)
    topk_err = int(max_over_ranks(float(topk_err), world))

    cpu = None
    if rank == 0 and not args.skip_cpu:  # after the GPU work, at every N (rank 0's host cores)
        cpu = cpu_baseline()
        for key, ck in (("config0_fedavg_10x417482", "aggregation_config0_fedavg_10x417482"),
                        ("config0_fedavg_10x417482", "aggregation_config0_host_server"),
                        ("config1_quant8_10x417482", "config2_quant8_10x417482"),
                        ("config2_topk1pct_25M", "config3_topk1pct_25M"),
                        ("config3_round_8x25M", "config4_codec_plus_rccl_reduce_25M"),
                        ("config0_compressed_round_stacked", "compressed_round_config0")):
            if ck in extra and key in cpu["configs"]:
                extra[ck]["cpu_torch"] = dict(cpu["configs"][key], threads=cpu["configs"]["threads"])

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": "configs[4]: 1 GiB fp32 delta per client, stacked top-k 1% -> 8-bit standard "
                            "dithering (s=127, p=inf, philox), encode+decode, device-resident",
                "D": D,
                "K": K,
                "bytes_per_step_per_client": stacked_bytes(D, K),
                "parallelism": f"one client per GPU x{world}",
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            "topk_err": topk_err,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    ok = topk_err == 0 and (rank != 0 or parity is None or parity["ok"])
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    if not ok:
        print(f"bench.py: self-check failed on rank {rank}: topk_err={topk_err}, parity={parity}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
