"""A/B of the single-client sample size (calibration builds diag/lib_s16.so, lib_s8.so: -DFLC_SAMPLE_CAP_DIAG) against
the 32 K default: configs[2] (25M top-k 1 %, encode + decode), a 1 M stacked encode and the 1 GiB headline step, one
child process per library, two alternating rounds."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, time, torch
sys.path.insert(0, %r)
from fl_sim_amd import codec
g = torch.Generator(device="cuda").manual_seed(0)
def tm(fn, reps):
    for i in range(10):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / reps
X3 = torch.randn(25_000_000, generator=g, device="cuda") * 1e-3
o3 = torch.empty_like(X3)
def c2(i):
    idx, val, tiles = codec.topk_encode(X3, 250_000, with_tiles=True)
    codec.sparse_decode(idx, val, X3.numel(), out=o3, tiles=tiles)
X1 = torch.randn(1_000_000, generator=g, device="cuda") * 1e-3
x = torch.randn(1 << 28, generator=g, device="cuda") * 1e-3
out = torch.empty_like(x)
def hl(i):
    codec.stacked_decode(codec.stacked_encode(x, (1 << 28) // 100, 127, seed=0, counter=i), out=out)
for _ in range(50):
    hl(0)
r = (tm(c2, 200), tm(lambda i: codec.stacked_encode(X1, 10_000, 127, seed=0, counter=i), 300), tm(hl, 40))
ok = codec.topk_status() == 0
print(f"{sys.argv[1]:5s} configs[2] {r[0]:6.1f} us   1M stacked encode {r[1]:5.1f} us   headline {r[2]:6.1f} us   err-free {ok}", flush=True)
""" % ROOT
for rnd in range(2):
    for v in ["main"] + sys.argv[1:]:
        env = dict(os.environ)
        if v != "main":
            env["FLC_LIB"] = os.path.join(ROOT, "diag", f"lib_{v}.so")
        r = subprocess.run([sys.executable, "-c", CHILD, v], env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-1500:], flush=True)
        if r.returncode:
            sys.exit(r.returncode)
