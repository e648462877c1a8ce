"""The headline decode with one 1024-output tile per wave (FLC_DECODE_NT1=1, 4 KB of output per workgroup) against the
default two tiles per wave (8 KB): decode alone and the whole step, each setting in its own child process (the knob is
read once per process), two alternating rounds; the one-tile output is checked equal to the default's."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, torch
sys.path.insert(0, %r)
from fl_sim_amd import codec
n = 1 << 28
k = n // 100
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1234)) * 1e-3
out = torch.empty_like(x)
pkt = codec.stacked_encode(x, k, 127, seed=1, counter=0)
c = [0]
def step():
    c[0] += 1
    p = codec.stacked_encode(x, k, 127, seed=1, counter=c[0])
    codec.stacked_decode(p, out=out)
def tm(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3
for _ in range(100):
    step()
d = tm(lambda: codec.stacked_decode(pkt, out=out))
codec.stacked_decode(pkt, out=out)
torch.save(out[:1 << 24].cpu(), "/tmp/dec_%%s.pt" %% sys.argv[1])
s = tm(step)
print(f"NT1={sys.argv[1]}: decode {d:6.1f} us, step {s:6.1f} us", flush=True)
""" % ROOT

for rnd in range(2):
    for v in ("0", "1"):
        env = dict(os.environ, FLC_DECODE_NT1=v)
        r = subprocess.run([sys.executable, "-c", CHILD, v], env=env, capture_output=True, text=True, timeout=200)
        print(r.stdout.strip() or r.stderr[-1500:], flush=True)
        if r.returncode:
            sys.exit(r.returncode)
import torch  # noqa: E402

print("outputs equal:", torch.equal(torch.load("/tmp/dec_0.pt"), torch.load("/tmp/dec_1.pt")))
