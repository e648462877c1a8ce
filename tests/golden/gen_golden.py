"""Generate tests/golden/*.npz by running the REFERENCE implementation (wenh06/fl-sim) in this container.

Runs only where /root/reference exists (never on the GPU box).  Nothing of the reference is copied:
the codec module is imported from its file path, and the aggregation methods are compiled from the
reference's own source text at run time (the full ``fl_sim`` package does not import here: torch_ecg
and other dependencies are absent).  Only inputs and outputs are written.

Codec fixtures (``codec_*.npz``): for each case the inputs (or, for large vectors, the seeded recipe
and a checksum), the seed given to ``random.seed`` / ``np.random.seed`` immediately before the call
(fl_sim/utils/misc.py:210-211 ``set_seed``), the reference output (full, or SHA-256 for large ones),
the send statistics, and the next value of each global stream after the call (stream lock-step).

Aggregation fixtures (``agg_*.npz``): FedOptServer.update (avg/adam/yogi/adagrad), avg_parameters
(size_aware x inertia) and update_gradients on small model shapes (full arrays) and on the
cnn_femmist_tiny shapes of config 1 (SHA-256 of the outputs).

Usage:  python tests/golden/gen_golden.py
"""

from __future__ import annotations

import ast
import hashlib
import importlib.util
import os
import random
import sys
import types
from pathlib import Path
from typing import Any, Dict, Iterable, List, Sequence

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

CONFIG1_SHAPES = [(16, 1, 5, 5), (16,), (32, 16, 5, 5), (32,), (256, 1568), (256,), (10, 256), (10,)]
SMALL_SHAPES = [(4, 1, 3, 3), (4,), (8, 4, 3, 3), (8,), (64, 49), (64,), (10, 64), (10,)]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def load_reference_compressors():
    spec = importlib.util.spec_from_file_location("ref_compressors", REF / "fl_sim/compressors/compressors.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_input(D: int, seed: int, zero_frac: float = 0.05, scale: float = 1e-3) -> np.ndarray:
    """Seeded synthetic delta that does NOT touch the global random streams."""
    g = np.random.default_rng(10_000 + seed * 7919 + D)
    x = (g.standard_normal(D) * scale).astype(np.float32)
    if D > 1:
        x[g.random(D) < zero_frac] = 0.0
    return x


def special_inputs() -> Dict[str, np.ndarray]:
    f = np.float32
    return {
        "ties": np.array([1, 3, 3, 3, 2, 3, 0, -1, 3, 2], dtype=f),
        "signed": np.array([-3.5, 1.5, 0.25, -0.0, 0.0, 2.0, -7.0, 1.5], dtype=f),
        "nan": np.array([0.5, np.nan, -1.0, 2.0, np.nan, 0.0, -0.0, 1.0], dtype=f),
        "zeros_pm": np.array([0.0, -0.0, 0.0, 1e-30, -0.0, -1e-30, 0.0], dtype=f),
        "powers2": np.array([1.0, -2.0, 0.5, 0.25, -0.125, 1024.0, 2.0**-20, 3.0], dtype=f),
        "subnormal": np.array([1e-40, -3e-42, 1e-45, 2.0**-126, -(2.0**-127), 0.1], dtype=f),
    }


def run_codec(ref, make, x: np.ndarray, seed: int):
    c = ref.Compressor()
    make(c)
    random.seed(seed)
    np.random.seed(seed)
    out = c.compressVector(x)
    rec = {
        "send": np.float64(c.last_need_to_send_advance),
        "total_in": np.float64(c.total_input_components),
        "next_random": np.float64(random.random()),
        "next_np": np.float64(np.random.random_sample()),
    }
    return out, rec


def codec_cases(ref):
    idn = lambda: (lambda c: c.makeIdenticalCompressor())  # noqa: E731

    def std(L, p, fp64=False):
        def mk(c):
            nc = ref.Compressor("norm")
            nc.makeIdenticalCompressor()
            (c.makeStandardDitheringFP64 if fp64 else c.makeStandardDitheringFP32)(L, nc, p)

        return mk

    cases = {
        "identical": idn(),
        "lazy_p03": lambda c: c.makeLazyCompressor(0.3),
        "lazy_p09": lambda c: c.makeLazyCompressor(0.9),
        "natural32": lambda c: c.makeNaturalCompressorFP32(),
        "natural64": lambda c: c.makeNaturalCompressorFP64(),
        "natdither32_s8_inf": lambda c: c.makeNaturalDitheringFP32(8, 100, np.inf),
        "natdither64_s3_p2": lambda c: c.makeNaturalDitheringFP64(3, 100, 2),
        "stddither32_s8_inf": std(8, np.inf),
        "stddither64_s4_inf": std(4, np.inf, fp64=True),
    }
    for L in (1, 3, 4, 7, 8, 10):
        for p, pn in ((np.inf, "inf"), (2, "p2")):
            cases[f"std_L{L}_{pn}"] = std(L, p)
    return cases


def gen_codecs(ref):
    cases = codec_cases(ref)
    store: Dict[str, Any] = {}
    big = 65537
    for name, mk in cases.items():
        sizes = (1, 7, 4096, big) if not name.startswith("std_L") else (7, 4096)
        for D in sizes:
            for seed in (0, 1, 42):
                if D == big and seed != 0:
                    continue
                x = make_input(D, seed)
                out, rec = run_codec(ref, mk, x, seed)
                key = f"{name}|{D}|{seed}"
                store[key + "|sha_x"] = np.array(sha(x))
                if D <= 4096:
                    store[key + "|x"] = x
                    store[key + "|out"] = out
                store[key + "|sha_out"] = np.array(sha(out))
                for k, v in rec.items():
                    store[key + "|" + k] = np.array(v)
    # special vectors (ties, NaN, signed zeros, powers of two, subnormals)
    for sname, x in special_inputs().items():
        for name in ("identical", "natural32", "stddither32_s8_inf", "natdither32_s8_inf"):
            if name != "identical" and sname == "nan":
                continue  # the reference raises or propagates NaN through the norm; covered in tests
            out, rec = run_codec(ref, cases[name], x, 3)
            key = f"{name}|special:{sname}|3"
            store[key + "|x"] = x
            store[key + "|out"] = out
            for k, v in rec.items():
                store[key + "|" + k] = np.array(v)
    np.savez_compressed(OUT / "codec_dense.npz", **store)
    print("codec_dense.npz:", len(store), "arrays")


def gen_sparse(ref):
    store: Dict[str, Any] = {}
    for D, K in ((7, 3), (4096, 41), (4096, 1), (65537, 655), (100, 0), (100, 100), (100, 150)):
        for seed in (0, 1, 42):
            x = make_input(D, seed)
            for name, mk in (
                ("topk", lambda c: c.makeTopKCompressor(K, D)),
                ("randk", lambda c: c.makeRandKCompressor(max(K, 1), D)),
            ):
                if name == "randk" and K > D:
                    continue
                out, rec = run_codec(ref, mk, x, seed)
                key = f"{name}|{D}|{K}|{seed}"
                store[key + "|sha_x"] = np.array(sha(x))
                if D <= 4096:
                    store[key + "|x"] = x
                    store[key + "|out"] = out
                store[key + "|sha_out"] = np.array(sha(out))
                for k, v in rec.items():
                    store[key + "|" + k] = np.array(v)
    for sname, x in special_inputs().items():
        for K in (1, 3, len(x) - 1):
            out, rec = run_codec(ref, lambda c: c.makeTopKCompressor(K, len(x)), x, 5)
            key = f"topk|special:{sname}|{K}|5"
            store[key + "|x"] = x
            store[key + "|out"] = out
            for k, v in rec.items():
                store[key + "|" + k] = np.array(v)
    # adaptive random: one index drawn with p = |x| / sum|x| (legacy np.random.choice)
    for D in (7, 4096):
        for seed in (0, 1, 42):
            x = make_input(D, seed, zero_frac=0.0)
            out, rec = run_codec(ref, lambda c: c.makeAdaptiveRandomCompressor(D), x, seed)
            key = f"adaptive|{D}|{seed}"
            store[key + "|x"] = x
            store[key + "|out"] = out
            for k, v in rec.items():
                store[key + "|" + k] = np.array(v)
    np.savez_compressed(OUT / "codec_sparse.npz", **store)
    print("codec_sparse.npz:", len(store), "arrays")


# ------------------------------------------------------------------------------------------- aggregation
def reference_methods() -> Dict[str, types.FunctionType]:
    """Compile the reference's own aggregation method bodies from its source text."""
    import typing

    from torch.nn.parameter import Parameter

    ns: Dict[str, Any] = {"torch": torch, "Parameter": Parameter, "np": np}
    ns.update({k: getattr(typing, k) for k in ("Any", "Dict", "Iterable", "List", "Optional", "Sequence", "Tuple", "Union")})
    wanted = {
        "fl_sim/nodes.py": ("Server", ("add_parameters", "avg_parameters", "update_gradients")),
        "fl_sim/algorithms/fedopt/_fedopt.py": (
            "FedOptServer",
            ("update", "update_avg", "update_adagrad", "update_yogi", "update_adam"),
        ),
    }
    fns: Dict[str, types.FunctionType] = {}
    for rel, (cls, names) in wanted.items():
        src = (REF / rel).read_text()
        tree = ast.parse(src)
        for node in tree.body:
            if isinstance(node, ast.ClassDef) and node.name == cls:
                for item in node.body:
                    if isinstance(item, ast.FunctionDef) and item.name in names:
                        item.decorator_list = []
                        mod = ast.Module(body=[item], type_ignores=[])
                        code = compile(mod, f"{REF / rel}:{item.lineno}", "exec")
                        local: Dict[str, Any] = {}
                        exec(code, ns, local)
                        fns[item.name] = local[item.name]
    missing = {n for _, (_, ns_) in wanted.items() for n in ns_} - set(fns)
    assert not missing, missing
    return fns


def make_model(shapes, seed):
    g = torch.Generator().manual_seed(seed)
    m = torch.nn.Module()
    for i, s in enumerate(shapes):
        m.register_parameter(f"p{i}", torch.nn.Parameter(torch.randn(s, generator=g) * 0.1))
    return m


def make_msgs(shapes, n, seed, key):
    g = torch.Generator().manual_seed(seed)
    return [
        {"client_id": i, "train_samples": 100 * (i + 1), "metrics": {}, key: [torch.randn(s, generator=g) * 1e-3 for s in shapes]}
        for i in range(n)
    ]


def gen_aggregation():
    fns = reference_methods()

    class FakeServer:
        pass

    for name, fn in fns.items():
        setattr(FakeServer, name, fn)

    store: Dict[str, Any] = {}
    for tag, shapes in (("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)):
        full = tag == "small"

        def put(key, tensors):
            flat = torch.cat([t.detach().reshape(-1) for t in tensors]).numpy()
            store[key + "|sha"] = np.array(sha(flat))
            if full:
                store[key + "|out"] = flat

        # FedOptServer.update for each server optimiser
        for opt, lr, betas, tau in (("avg", 1, (0, 1), 1), ("adam", 0.01, (0.9, 0.99), 1e-3),
                                    ("yogi", 0.01, (0.9, 0.99), 1e-3), ("adagrad", 0.05, (0.0, 0.99), 1e-3)):
            s = FakeServer()
            s.model = make_model(shapes, 1)
            s.device = torch.device("cpu")
            s.config = types.SimpleNamespace(optimizer=opt, lr=lr, betas=betas, tau=tau)
            g = torch.Generator().manual_seed(2)
            s.delta_parameters = [torch.randn(sh, generator=g) * 1e-3 for sh in shapes]
            s.v_parameters = None if opt == "avg" else [torch.rand(sh, generator=g) * 1e-4 + 1e-6 for sh in shapes]
            s._received_messages = make_msgs(shapes, 10, 3, "delta_parameters")
            s.update()
            put(f"fedopt_{opt}_{tag}|theta", list(s.model.parameters()))
            put(f"fedopt_{opt}_{tag}|delta", s.delta_parameters)
            if s.v_parameters is not None:
                put(f"fedopt_{opt}_{tag}|v", s.v_parameters)
        # avg_parameters
        for size_aware in (False, True):
            for inertia in (0.0, 0.3):
                s = FakeServer()
                s.model = make_model(shapes, 4)
                s.device = torch.device("cpu")
                s._received_messages = make_msgs(shapes, 10, 5, "parameters")
                s.avg_parameters(size_aware=size_aware, inertia=inertia)
                put(f"avgp_{int(size_aware)}_{inertia}_{tag}|theta", list(s.model.parameters()))
        # update_gradients
        s = FakeServer()
        s.model = make_model(shapes, 6)
        s.device = torch.device("cpu")
        s._received_messages = make_msgs(shapes, 10, 7, "gradients")
        s.update_gradients()
        put(f"gradients_{tag}|grad", [p.grad for p in s.model.parameters()])
    np.savez_compressed(OUT / "agg.npz", **store)
    print("agg.npz:", len(store), "arrays")


def main():
    if not REF.exists():
        print("reference not present; nothing to do", file=sys.stderr)
        return 1
    torch.set_num_threads(1)
    ref = load_reference_compressors()
    gen_codecs(ref)
    gen_sparse(ref)
    gen_aggregation()
    return 0


if __name__ == "__main__":
    sys.exit(main())
