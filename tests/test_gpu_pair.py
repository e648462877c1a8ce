"""The paired pass of the top-k encoders (topk.hip filter_phase, opt-in with FLC_PAIR=1): blocks 2j and 2j + 1 stream
their joint range from both ends and claim the middle steps at run time, so each block's range is decided during the
pass.  The packets must not depend on it: a child process with FLC_PAIR=1 (the switch is read once per process)
encodes the same inputs as this one, and every packet must be bit-identical — at the headline's shape, with the
candidates past LDS (the HBM overflow of a reverse block, read back top down), at the delta-fused encoder's shape, and
with a partial last pair (static ranges)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, sys, torch
sys.path.insert(0, sys.argv[1])
from fl_sim_amd import codec
out = []
def h(*ts):
    m = hashlib.sha256()
    for t in ts:
        m.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return m.hexdigest()
for n, frac, skew in ((1 << 26, 0.01, False), (32 << 20, 0.15, False), (24 << 20, 0.01, True), (50_000_017, 0.01, False)):
    g = torch.Generator(device="cuda").manual_seed(n % 997)
    x = torch.randn(n, generator=g, device="cuda") * 1e-3
    if skew:  # the largest values in one region: some blocks far past the LDS's candidates
        x[: n // 16] += 1.0
    k = int(n * frac)
    p = codec.stacked_encode(x, k, 127, seed=3, counter=5)
    i, v = codec.topk_encode(x, k)
    out.append(h(p.idx, p.codes, p.norm, p.tiles, i, v))
sizes = [(1 << 20) + 3 * i for i in range(31)] + [1 << 20]
g = torch.Generator(device="cuda").manual_seed(7)
glob = [torch.randn(s, generator=g, device="cuda") for s in sizes]
loc = [t + torch.randn(t.shape, generator=g, device="cuda") * 1e-3 for t in glob]
n = sum(sizes)
p = codec.stacked_encode_delta(loc, glob, n // 100, 127, seed=1, counter=2)
out.append(h(p.idx, p.codes, p.norm, p.tiles))
print("\n".join(out))
print("err", sum(codec.topk_status_all().values()))
"""


def _run(pair: str) -> list:
    env = dict(os.environ, FLC_PAIR=pair)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln and not ln.startswith("/opt")]
    assert lines[-1] == "err 0", lines[-1]
    return lines[:-1]


def test_paired_pass_packets_equal_static_ranges():
    torch.cuda.synchronize()
    assert _run("1") == _run("0")
