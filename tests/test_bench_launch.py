"""bench.py's N-rank launcher (CPU rehearsal with gloo; no GPU work).

`python bench.py --gpus N` without a torch.distributed environment must start N ranks itself (one
child launcher, never an exec of this process), every rank must check that the world it joined has
exactly N ranks, and a mismatch must exit non-zero instead of reporting a different GPU count.
"""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def _json_line(out: str) -> dict:
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_launcher_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--launch-check"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1] and line["distinct_pids"] == 2


def test_world_size_mismatch_is_refused():
    # a world of 1 joined with --gpus 2: no launch (WORLD_SIZE is set), refuse
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--launch-check"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 3
    assert "refusing" in r.stderr


def test_launcher_world_mismatch_under_torchrun():
    # torchrun with 2 ranks, bench asked for 3: every rank refuses, the launcher reports failure
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", "0", BENCH, "--gpus", "3",
                        "--backend", "gloo", "--launch-check"],
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode != 0


def test_gloo_backend_needs_launch_check():
    r = subprocess.run([sys.executable, BENCH, "--backend", "gloo"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
