"""CPU tests of the C-ABI library: it loads, exports every symbol include/flcodec.h declares, and its
host-side logic (compat RNG, argument validation) is right.  No GPU compute is launched here."""

import ctypes
import os
import random
import re

import numpy as np
import pytest

from fl_sim_amd import _lib, rng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "flcodec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(flc_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_abi_version():
    lib = _lib.load()
    assert lib.flc_abi_version() == 1
    assert os.path.isfile(_lib.LIB_PATH)


def test_every_header_symbol_is_exported_and_bound():
    names = header_functions()
    assert len(names) >= 20
    lib = _lib.load()
    for n in names:
        assert hasattr(lib, n), f"{n} declared in flcodec.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature in _lib.py"
    assert set(_lib.SIGNATURES) == set(names)


def test_error_reporting():
    with pytest.raises(_lib.FlcError, match="levels"):
        _lib.call("flc_quant_encode", 1, 1, 8, 0, 200, 8, 1, 0, 0, None, 1, None, 1, 1, None)
    with pytest.raises(_lib.FlcError, match="0 < k < n"):
        _lib.call("flc_topk_encode", 16, 10, 10, 1, 1, 1, 1, None)


@pytest.mark.parametrize("seed", [0, 1, 42, 12345])
@pytest.mark.parametrize("n", [0, 1, 311, 312, 313, 5000])
def test_python_random_lockstep(seed, n):
    random.seed(seed)
    expect = [random.random() for _ in range(n)]
    after = random.random()
    random.seed(seed)
    got = rng.python_random_doubles(n)
    assert got.tolist() == expect
    assert random.random() == after


@pytest.mark.parametrize("seed", [0, 3, 42])
@pytest.mark.parametrize("D,K", [(1, 1), (7, 3), (100, 10), (4097, 41), (1000, 1500)])
def test_numpy_shuffle_lockstep(seed, D, K):
    np.random.seed(seed)
    S = np.arange(D)
    np.random.shuffle(S)
    expect = S[:K]
    after = np.random.random_sample()
    np.random.seed(seed)
    got = rng.numpy_shuffle_prefix(D, K)
    assert np.array_equal(got, expect)
    assert np.random.random_sample() == after


def test_workspace_sizes_monotone():
    a = _lib.size("flc_topk_workspace_size", 1 << 20, 1 << 10)
    b = _lib.size("flc_topk_workspace_size", 1 << 22, 1 << 12)
    assert 0 < a < b
    assert _lib.size("flc_quant_workspace_size", 10, 417482) > 0
    assert _lib.size("flc_natural_workspace_size", 417482) > 0


def test_topk_status_plumbing_without_gpu(monkeypatch):
    """flc_topk_status validates its arguments before any HIP call; codec raises when the word is set."""
    from fl_sim_amd import _lib, codec

    lib = _lib.load()
    assert lib.flc_topk_status(None, None, 1, None) == 1  # FLC_EINVAL
    assert "flc_topk_status" in lib.flc_last_error().decode()
    monkeypatch.setattr(codec, "TOPK_CHECK", True)
    seen = []
    monkeypatch.setattr(codec, "_status", lambda device, kinds, reset=True: seen.append(tuple(kinds)) or 4)
    with pytest.raises(_lib.FlcError, match="top-k encode.*spin timeout"):
        codec._after_encode(None)
    # the one-launch quantizer's exchange is checked too (its own workspace kind)
    with pytest.raises(_lib.FlcError, match="quantizer.*spin timeout"):
        codec._after_encode(None, ("quant",))
    assert seen == [codec._TOPK_KINDS, ("quant",)]
    monkeypatch.setattr(codec, "_status", lambda device, kinds, reset=True: 0)
    codec._after_encode(None)  # clean word: no error
    codec._after_encode(None, ("quant",))


def test_stacked_encode_delta_validates_without_gpu():
    """flc_stacked_encode_delta rejects bad tensor tables before touching the device."""
    from fl_sim_amd import _lib

    lib = _lib.load()
    P = ctypes.c_void_p * 2
    S = ctypes.c_int64 * 2
    good = P(16, 32)
    assert lib.flc_stacked_encode_delta(None, None, None, 0, 1, 127, 0, 0, 16, 16, 16, None, 16, 1 << 30, None) == 1
    # misaligned tensor pointer
    rc = lib.flc_stacked_encode_delta(ctypes.cast(P(18, 32), ctypes.c_void_p), ctypes.cast(good, ctypes.c_void_p),
                                      ctypes.cast(S(100, 100), ctypes.c_void_p), 2, 10, 127, 0, 0, 16, 16, 16, None, 16,
                                      1 << 30, None)
    assert rc == 1 and "aligned" in lib.flc_last_error().decode()
    # k out of range
    rc = lib.flc_stacked_encode_delta(ctypes.cast(good, ctypes.c_void_p), ctypes.cast(good, ctypes.c_void_p),
                                      ctypes.cast(S(100, 100), ctypes.c_void_p), 2, 200, 127, 0, 0, 16, 16, 16, None, 16,
                                      1 << 30, None)
    assert rc == 1 and "0 < k < n" in lib.flc_last_error().decode()
    assert lib.flc_stacked_encode_delta_workspace_size(1000, 10, 8) > lib.flc_topk_workspace_size(1000, 10)


def test_stacked_encode_batch_validates_without_gpu():
    """flc_stacked_encode_batch rejects bad client tables before touching the device; its workspace grows with the
    client count."""
    from fl_sim_amd import _lib

    lib = _lib.load()
    P = ctypes.c_void_p * 2
    U = ctypes.c_uint64 * 2
    c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    good, seeds = P(16, 32), U(1, 2)
    assert lib.flc_stacked_encode_batch(None, 2, 100, 10, 127, None, 0, None, None, None, None, 16, 1 << 30,
                                        None) == 1
    rc = lib.flc_stacked_encode_batch(c(good), 0, 100, 10, 127, c(seeds), 0, c(good), c(good), c(good), None, 16,
                                      1 << 30, None)
    assert rc == 1 and "bad arguments" in lib.flc_last_error().decode()
    rc = lib.flc_stacked_encode_batch(c(good), 2, 100, 10, 200, c(seeds), 0, c(good), c(good), c(good), None, 16,
                                      1 << 30, None)
    assert rc == 1 and "levels" in lib.flc_last_error().decode()
    rc = lib.flc_stacked_encode_batch(c(P(16, 40)), 2, 100, 10, 127, c(seeds), 0, c(good), c(good), c(good), None, 16,
                                      1 << 30, None)  # client 1's input not 16-B aligned
    assert rc == 1 and "aligned" in lib.flc_last_error().decode()
    rc = lib.flc_stacked_encode_batch(c(good), 2, 100, 100, 127, c(seeds), 0, c(good), c(good), c(good), None, 16,
                                      1 << 30, None)
    assert rc == 1 and "0 < k < n" in lib.flc_last_error().decode()
    rc = lib.flc_stacked_encode_batch(c(good), 2, 100, 10, 127, c(seeds), 0, c(P(16, 0)), c(good), c(good), None, 16,
                                      1 << 30, None)
    assert rc == 1 and "null output of client 1" in lib.flc_last_error().decode()
    a = lib.flc_stacked_encode_batch_workspace_size(1 << 20, 1 << 10, 2)
    b = lib.flc_stacked_encode_batch_workspace_size(1 << 20, 1 << 10, 8)
    assert 0 < a < b


def test_stacked_encode_delta_batch_validates_without_gpu():
    from fl_sim_amd import _lib

    lib = _lib.load()
    P2, P4 = ctypes.c_void_p * 2, ctypes.c_void_p * 4
    c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    sizes, seeds = (ctypes.c_int64 * 2)(100, 100), (ctypes.c_uint64 * 2)(1, 2)
    good2, good4 = P2(16, 32), P4(16, 32, 48, 64)
    args = lambda loc, glob, k: (c(loc), c(glob), c(sizes), 2, 2, k, 127, c(seeds), 0, c(good2), c(good2), c(good2),  # noqa: E731
                                 None, 16, 1 << 30, None)
    assert lib.flc_stacked_encode_delta_batch(None, None, None, 2, 2, 10, 127, None, 0, None, None, None, None, 16,
                                              1 << 30, None) == 1
    assert lib.flc_stacked_encode_delta_batch(*args(P4(16, 32, 50, 64), good2, 10)) == 1  # client 1's tensor 0
    assert "local tensor 0 of client 1" in lib.flc_last_error().decode()
    assert lib.flc_stacked_encode_delta_batch(*args(good4, P2(16, 34), 10)) == 1
    assert "global tensor 1" in lib.flc_last_error().decode()
    assert lib.flc_stacked_encode_delta_batch(*args(good4, good2, 200)) == 1
    assert "0 < k < n" in lib.flc_last_error().decode()
    assert (lib.flc_stacked_encode_delta_batch_workspace_size(200, 2, 8, 2) >
            lib.flc_stacked_encode_batch_workspace_size(200, 2, 8))


def test_topk_encode_batch_validates_without_gpu():
    from fl_sim_amd import _lib

    lib = _lib.load()
    P = ctypes.c_void_p * 2
    c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    assert lib.flc_topk_encode_batch(None, 2, 100, 10, None, None, None, 16, 1 << 30, None) == 1
    assert lib.flc_topk_encode_batch(c(P(16, 40)), 2, 100, 10, c(P(16, 32)), c(P(16, 32)), None, 16, 1 << 30, None) == 1
    assert "aligned" in lib.flc_last_error().decode()
    assert lib.flc_topk_encode_batch(c(P(16, 32)), 2, 100, 10, c(P(16, 32)), c(P(16, 0)), None, 16, 1 << 30, None) == 1
    assert "null output of client 1" in lib.flc_last_error().decode()
    assert lib.flc_topk_encode_batch_workspace_size(1000, 10, 4) == lib.flc_stacked_encode_batch_workspace_size(1000, 10, 4)


def test_rccl_entries_validate_without_gpu():
    """The RCCL entries (flc_comm_* / flc_rccl_*) check their arguments before RCCL is touched; the unique id is
    RCCL's 128 bytes."""
    import ctypes

    lib = _lib.load()
    assert _lib.size("flc_comm_id_bytes") == 128
    h = ctypes.c_void_p()
    assert lib.flc_comm_init(None, 1, 0, -1, ctypes.byref(h)) == 1
    uid = ctypes.create_string_buffer(128)
    assert lib.flc_comm_init(ctypes.cast(uid, ctypes.c_void_p), 2, 2, -1, ctypes.byref(h)) == 1  # rank >= nranks
    n, r = ctypes.c_int(), ctypes.c_int()
    assert lib.flc_comm_size(None, ctypes.byref(n), ctypes.byref(r)) == 1
    assert lib.flc_rccl_reduce(None, None, 5, 0, None, None) == 1
    assert lib.flc_rccl_allreduce(None, None, 5, None, None) == 1
    assert lib.flc_rccl_allgather(None, None, 0, None, None) == 1
    assert lib.flc_comm_destroy(None) == 0  # destroying nothing is a no-op


def test_f64_entries_validate_without_gpu():
    """The float64 forms (f64.hip, adaptive.hip) reject bad arguments before touching the device, and the top-k
    workspace grows with k's candidate segments."""
    lib = _lib.load()
    assert lib.flc_topk_dense_f64(16, 100, 0, 16, 16, 1 << 30, None) == 1
    assert "0 < k < n" in lib.flc_last_error().decode()
    assert lib.flc_topk_dense_f64(24, 100, 5, 16, 16, 1 << 30, None) == 1
    assert "aligned" in lib.flc_last_error().decode()
    assert lib.flc_quant_f64(16, 100, 0, 128, 16, 0, 0, None, 16, 16, None, 16, 1 << 30, None) == 1
    assert "levels" in lib.flc_last_error().decode()
    assert lib.flc_quant_f64(16, 100, 7, 8, 16, 0, 0, None, 16, 16, None, 16, 1 << 30, None) == 1
    assert lib.flc_quant_norm_f64(16, 100, 3, 16, 16, 1 << 30, None) == 4  # p = 3: FLC_EUNSUPPORTED
    assert lib.flc_natural_f64(16, 100, 0, 0, None, None, None, 16, 1 << 30, None) == 1  # neither codes nor out
    assert lib.flc_adaptive_select_f64(16, 100, 1.5, 16, 16, 16, 1 << 30, None) == 1  # u outside [0, 1)
    assert lib.flc_adaptive_stats(None, 1 << 30, 100, 16, None) == 1  # no workspace
    assert lib.flc_adaptive_stats(16, 8, 100, 16, None) == 3  # workspace too small: FLC_EWORKSPACE
    assert lib.flc_f64_workspace_size(1 << 24, 1 << 17) > lib.flc_f64_workspace_size(1 << 24, 0)
    # small n: the selection state only (no candidate segments)
    assert 0 < lib.flc_f64_workspace_size(1000, 10) - lib.flc_f64_workspace_size(1000, 0) < 1 << 20


_STUB_RCCL = r"""
#include <string.h>
typedef struct { char internal[128]; } ncclUniqueId;
int ncclGetUniqueId(ncclUniqueId* id) { memset(id, 0x5a, sizeof(*id)); return 0; }
int ncclCommInitRank(void** c, int n, ncclUniqueId id, int r) { return 5; }
int ncclCommDestroy(void* c) { return 0; }
int ncclReduce(const void* a, void* b, unsigned long n, int t, int o, int root, void* c, void* s) { return 5; }
int ncclAllReduce(const void* a, void* b, unsigned long n, int t, int o, void* c, void* s) { return 5; }
int ncclAllGather(const void* a, void* b, unsigned long n, int t, void* c, void* s) { return 5; }
const char* ncclGetErrorString(int e) { return "stub rccl"; }
int ncclCommCount(void* c, int* n) { *n = 1; return 0; }
int ncclCommUserRank(void* c, int* r) { *r = 0; return 0; }
"""

_STUB_DRIVER = r"""
import ctypes, sys
ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)  # the stub's nccl* symbols in the global namespace first
from fl_sim_amd import _lib
lib = _lib.load()
uid = ctypes.create_string_buffer(128)
assert lib.flc_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)) == 0, lib.flc_last_error()
assert uid.raw == b"\x5a" * 128, "the id did not come from the global-namespace RCCL"
print(lib.flc_comm_rccl_origin().decode())
"""


def test_rccl_found_in_global_namespace(tmp_path):
    """RCCL symbols already in the process's global namespace (glibc's RTLD_DEFAULT is a null handle) are
    the ones used — no second RCCL is loaded.  A stub RCCL is loaded RTLD_GLOBAL in a fresh process first."""
    import shutil
    import subprocess
    import sys

    gcc = shutil.which("gcc") or shutil.which("cc")
    if gcc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "stub_rccl.c"
    src.write_text(_STUB_RCCL)
    so = tmp_path / "libstubnccl.so"
    subprocess.run([gcc, "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    env = dict(os.environ)
    env.pop("FLC_RCCL_LIB", None)
    env["PYTHONPATH"] = os.pathsep.join([ROOT, env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", _STUB_DRIVER, str(so)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == "global"


def test_model_fold_ctypes_checks_sizes(monkeypatch):
    """the ctypes form of model_fold checks theta / v sizes and the weight count (ValueError) before any
    pointer is taken, as the torch op does; a mismatch must never reach the kernel."""
    import torch

    from fl_sim_amd import codec

    monkeypatch.setattr(codec, "_MODEL_FOLD_OP", [None])
    monkeypatch.setattr(codec, "_PYFOLD", [None])
    d = [torch.zeros(5), torch.zeros(3)]
    msgs = [[torch.zeros(5), torch.zeros(3)]]
    with pytest.raises(ValueError, match="one weight per message"):
        codec.model_fold(d, msgs, [0.5, 0.5], 0)
    with pytest.raises(ValueError, match="theta"):
        codec.model_fold(d, msgs, [0.5], 0, theta=[torch.zeros(5), torch.zeros(4)])
    with pytest.raises(ValueError, match="v must"):
        codec.model_fold(d, msgs, [0.5], 0, theta=[torch.zeros(5), torch.zeros(3)], v=[torch.zeros(5)], opt="adam")


def test_pyfold_module_checks_without_gpu():
    """fl_sim_amd._flcfold (csrc/pyfold.cpp) loads and rejects what the fold does not take before anything runs: host
    tensors (TypeError, the callers' cue to move messages), count and size mismatches (ValueError)."""
    import torch

    from fl_sim_amd import _flcfold

    d = [torch.zeros(5), torch.zeros(3)]
    with pytest.raises(TypeError, match="HIP"):
        _flcfold.model_fold(d, [d], None, [0.5], 0, 0.0, None, None, 0, 1.0, 0.0, 0.0)
    with pytest.raises(ValueError, match="one weight per message"):
        _flcfold.model_fold(d, [d], None, [0.5, 0.5], 0, 0.0, None, None, 0, 1.0, 0.0, 0.0)
    _flcfold.model_fold([], [], None, [], 0, 0.0, None, None, 0, 1.0, 0.0, 0.0)  # nothing to fold


def _ring(ops):
    """Drive the batched encoders' pinned table ring bookkeeping (flc_ring_selftest, no device): ops are ("s",) to
    stage the next slot or ("d", slot, stream) to mark a slot done; returns [(slot, wait, event_slot)] per stage."""
    lib = _lib.load()
    flat = []
    for op in ops:
        flat += [0, 0, 0] if op[0] == "s" else [1, op[1], op[2]]
    n = len(ops)
    a = (ctypes.c_int32 * max(1, 3 * n))(*flat)
    out = (ctypes.c_int32 * max(1, 3 * n))()
    w = lib.flc_ring_selftest(a, n, out, n)
    assert w >= 0
    return [tuple(out[3 * i:3 * i + 3]) for i in range(w)]


def _lap(stream=1, skip_done=()):
    """One lap of 32 stage + done pairs on one stream (slots in `skip_done` staged but never done: an error return
    between stage_table and table_done)."""
    ops = []
    for s in range(32):
        ops.append(("s",))
        if s not in skip_done:
            ops.append(("d", s, stream))
    return ops


NONE, EVENT, DRAIN = 0, 1, 2


def test_table_ring_reuse_waits_for_the_covering_event():
    """Second lap on one stream: slot s waits for the event of slot s | 7 (recorded after it in the first lap)."""
    res = _ring(_lap() + _lap())
    assert [r[0] for r in res] == list(range(32)) * 2
    assert all(r[1] == NONE for r in res[:32])
    for s, (slot, wait, q) in enumerate(res[32:]):
        assert slot == s and wait == EVENT and q == (s | 7)


def test_table_ring_stage_without_done_never_trusts_a_stale_event():
    """Verdict r04 item 8: slot q = 7's stage in lap 2 fails before table_done.  In lap 3, slots 0..7 (covered by q in
    lap 2) must not wait on q's event from lap 1: they drain the device instead."""
    ops = _lap() + _lap(skip_done={7}) + _lap()
    res = _ring(ops)
    lap3 = res[64:]
    assert lap3[0][1] == DRAIN  # slot 0: q = 7 never completed its lap-2 use
    # after the drain every earlier use is complete: the next slots of the lap need no wait at all
    assert all(r[1] == NONE for r in lap3[1:8])
    # slots 8.. were staged in lap 2 *before* the drain: complete now, no wait either
    assert all(r[1] == NONE for r in lap3[8:32])


def test_table_ring_mixed_streams_drain():
    """A slot used on stream 2 whose covering slot ran on stream 1: the event does not cover it -> drain."""
    ops = []
    for s in range(32):
        ops += [("s",), ("d", s, 2 if s == 3 else 1)]
    ops += [("s",)] * 4
    res = _ring(ops)
    assert [r[1] for r in res[32:35]] == [EVENT, EVENT, EVENT]
    assert res[35][1] == DRAIN


def test_table_ring_event_from_an_earlier_lap_is_not_used():
    """Slot 7 done in lap 1 but its lap-2 stage never done; slot 0 of lap 2 done.  Reusing slot 0 in lap 3 must not
    take slot 7's lap-1 event (recorded before slot 0's lap-2 use)."""
    ops = _lap() + [("s",), ("d", 0, 1)]
    ops += [op for s in range(1, 32) for op in ([("s",)] if s == 7 else [("s",), ("d", s, 1)])]
    ops += [("s",)]
    res = _ring(ops)
    assert res[-1][0] == 0 and res[-1][1] == DRAIN
