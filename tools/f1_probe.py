"""f1: the delta-fused stacked encode (flc_stacked_encode_delta) at 1 GiB in 64 tensors, against the plain encode of
the flat delta: tensor sizes all multiples of 4 (every tensor's 16-B loads aligned) vs the bench's sizes (2^22 + i % 3:
most tensors start at a flat offset that is not a multiple of 4, so their loads are only 4-B aligned), each with the
global list allocated right after the local one (the bench's layout) and with the two interleaved."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fl_sim_amd import codec, _lib  # noqa: E402
import ctypes  # noqa: E402


def probe(name, fn, reps=20):
    """average duration of the named kernel over reps calls (live HIP-event probe)"""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.call("flc_probe_set", name.encode())
    _lib.call("flc_probe_read", None, None)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    t, c = ctypes.c_double(), ctypes.c_int64()
    _lib.call("flc_probe_read", ctypes.byref(t), ctypes.byref(c))
    _lib.call("flc_probe_set", None)
    return t.value / max(c.value, 1) * 1e3


def tm(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


g = torch.Generator(device="cuda").manual_seed(3)
for label, sizes in (("aligned", [1 << 22] * 64), ("bench_sizes", [(1 << 22) + (i % 3) for i in range(63)])):
    if len(sizes) == 63:
        sizes.append((1 << 28) - sum(sizes))
    n = sum(sizes)
    k = n // 100
    for layout in ("consecutive", "interleaved"):
        if layout == "consecutive":
            loc = [torch.randn(s, generator=g, device="cuda") for s in sizes]
            glo = [torch.randn(s, generator=g, device="cuda") for s in sizes]
        else:
            loc, glo = [], []
            for s in sizes:
                loc.append(torch.randn(s, generator=g, device="cuda"))
                glo.append(torch.randn(s, generator=g, device="cuda"))
        flat = codec.delta_flatten(loc, glo)
        t_plain = tm(lambda: codec.stacked_encode(flat, k, 127, seed=1, counter=2))
        t_fused = tm(lambda: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=2))
        print(f"{label:12s} {layout:12s} plain {t_plain:7.1f} us  fused {t_fused:7.1f} us  ratio {t_fused / t_plain:.3f}",
              flush=True)
        if os.environ.get("F1_KERNELS"):
            pk = {kn: probe(kn, lambda: codec.stacked_encode(flat, k, 127, seed=1, counter=2))
                  for kn in ("topk_sample", "stacked_encode")}
            fk = {kn: probe(kn, lambda: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=2))
                  for kn in ("topk_sample", "stacked_encode")}
            print("   kernels plain", {a: round(b, 1) for a, b in pk.items()}, "fused", {a: round(b, 1) for a, b in fk.items()},
                  flush=True)
        del loc, glo, flat
        torch.cuda.empty_cache()
