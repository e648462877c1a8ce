"""ctypes binding of the C ABI in ``include/flcodec.h`` (``fl_sim_amd/libflcodec.so``).

This is the binding a maintainer of the reference would add: plain pointers,
sizes and a ``hipStream_t``; no framework types cross the boundary.  The library is built in-tree by
``__graft_entry__.build()`` (``make -C fl_sim_amd/csrc``).  There is deliberately no fallback: if
the library is missing or fails to load, every codec call raises.
"""

from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

# FLC_LIB overrides the path (calibration builds under tools/ only)
LIB_PATH = os.environ.get("FLC_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libflcodec.so")

FLC_OK = 0
FLC_Q_STANDARD_DITHER = 0
FLC_Q_NATURAL_DITHER = 1
FLC_NORM_INF = 0
FLC_NORM_L2 = 2
FLC_OPT = {"avg": 0, "adagrad": 1, "yogi": 2, "adam": 3}
FLC_PROX_NONE, FLC_PROX_L1, FLC_PROX_SCALE = 0, 1, 2
FLC_SRV_FEDDYN, FLC_SRV_PFEDME = 1, 2

# name -> (restype, argtypes); must list every function declared in include/flcodec.h
SIGNATURES = {
    "flc_abi_version": (c_int, []),
    "flc_last_error": (c_char_p, []),
    "flc_workspace_init": (c_int, [c_void_p, c_size_t, c_void_p]),
    "flc_mt_random_doubles": (c_int, [POINTER(c_uint32), POINTER(c_int32), POINTER(c_double), c_int64]),
    "flc_np_shuffle_prefix": (c_int, [POINTER(c_uint32), POINTER(c_int32), c_int64, c_int64, POINTER(c_int32)]),
    "flc_quant_workspace_size": (c_size_t, [c_int64, c_int64]),
    "flc_quant_norm": (c_int, [c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_quant_encode": (
        c_int,
        [c_void_p, c_int64, c_int64, c_int, c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "flc_quant_encode_decode": (
        c_int,
        [c_void_p, c_int64, c_int64, c_int, c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "flc_quant_encode_auto": (
        c_int,
        [c_void_p, c_int64, c_int64, c_int, c_int, c_int, c_int, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "flc_quant_decode": (
        c_int, [c_void_p, c_int64, c_int64, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]
    ),
    "flc_count_consumers": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "flc_natural_workspace_size": (c_size_t, [c_int64]),
    "flc_natural_encode": (
        c_int, [c_void_p, c_int64, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_natural_decode": (c_int, [c_void_p, c_int64, c_float, c_int, c_void_p, c_void_p]),
    "flc_topk_workspace_size": (c_size_t, [c_int64, c_int64]),
    "flc_topk_status": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "flc_ring_selftest": (c_int, [POINTER(c_int32), c_int, POINTER(c_int32), c_int]),
    "flc_topk_encode": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_sparse_decode_workspace_size": (c_size_t, [c_int64]),
    "flc_sparse_decode": (
        c_int, [c_void_p, c_void_p, c_int64, c_float, c_int64, c_float, c_int, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_stacked_encode": (
        c_int,
        [c_void_p, c_int64, c_int64, c_int, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_size_t, c_void_p],
    ),
    "flc_stacked_encode_delta_workspace_size": (c_size_t, [c_int64, c_int64, c_int]),
    "flc_stacked_encode_delta": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_int, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "flc_stacked_encode_batch_workspace_size": (c_size_t, [c_int64, c_int64, c_int]),
    "flc_stacked_encode_batch": (
        c_int,
        [c_void_p, c_int, c_int64, c_int64, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "flc_topk_encode_batch_workspace_size": (c_size_t, [c_int64, c_int64, c_int]),
    "flc_topk_encode_batch": (
        c_int, [c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_stacked_encode_delta_batch_workspace_size": (c_size_t, [c_int64, c_int64, c_int, c_int]),
    "flc_stacked_encode_delta_batch": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "flc_stacked_decode": (
        c_int,
        [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64, c_float, c_int, c_void_p, c_void_p, c_size_t, c_void_p],
    ),
    "flc_tile_index": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "flc_topk_encode_tiled": (
        c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_sparse_decode_tiled": (
        c_int, [c_void_p, c_void_p, c_int64, c_float, c_int64, c_float, c_int, c_void_p, c_void_p, c_void_p]
    ),
    "flc_stacked_encode_tiled": (
        c_int,
        [c_void_p, c_int64, c_int64, c_int, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "flc_stacked_decode_tiled": (
        c_int,
        [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64, c_float, c_int, c_void_p, c_void_p, c_void_p],
    ),
    "flc_stacked_wire_layout": (c_size_t, [c_int64, c_int64, c_void_p]),
    "flc_stacked_fold_wires": (
        c_int,
        [c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int64, c_int64, c_int, c_int, c_void_p, c_void_p],
    ),
    "flc_fedopt_fold_records": (
        c_int,
        [c_void_p, c_void_p, c_int, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float,
         c_int, c_double, c_double, c_double, c_void_p],
    ),
    "flc_comm_id_bytes": (c_size_t, []),
    "flc_comm_rccl_origin": (c_char_p, []),
    "flc_comm_unique_id": (c_int, [c_void_p]),
    "flc_comm_init": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "flc_comm_size": (c_int, [c_void_p, c_void_p, c_void_p]),
    "flc_comm_destroy": (c_int, [c_void_p]),
    "flc_rccl_reduce": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "flc_rccl_allreduce": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_rccl_allgather": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_quant_status": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "flc_adaptive_workspace_size": (c_size_t, [c_int64]),
    "flc_adaptive_prepare": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_adaptive_select": (c_int, [c_void_p, c_int64, c_double, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_adaptive_prepare_f64": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_adaptive_select_f64": (
        c_int, [c_void_p, c_int64, c_double, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_adaptive_stats": (c_int, [c_void_p, c_size_t, c_int64, c_void_p, c_void_p]),
    "flc_copy": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_scale_div": (c_int, [c_void_p, c_int64, c_float, c_void_p, c_void_p]),
    "flc_randk_keys": (c_int, [c_int64, c_uint64, c_uint64, c_void_p, c_void_p]),
    "flc_randk_apply": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_float, c_void_p, c_void_p]),
    "flc_weighted_sum_f64": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int, c_double, c_void_p, c_void_p]),
    "flc_fedopt_step_f64": (
        c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_double, c_double, c_double, c_void_p]
    ),
    "flc_feddr_combine_f64": (
        c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_double, c_double, c_double, c_int, c_double, c_void_p]
    ),
    "flc_copy_f64": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_scale_div_f64": (c_int, [c_void_p, c_int64, c_double, c_void_p, c_void_p]),
    "flc_randk_apply_f64": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_double, c_void_p, c_void_p]),
    "flc_f64_workspace_size": (c_size_t, [c_int64, c_int64]),
    "flc_f64_status": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "flc_count_consumers_f64": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_natural_f64": (
        c_int, [c_void_p, c_int64, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    ),
    "flc_natural_decode_f64": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_quant_norm_f64": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_quant_f64": (
        c_int,
        [c_void_p, c_int64, c_int, c_int, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_size_t, c_void_p],
    ),
    "flc_quant_decode_f64": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "flc_topk_dense_f64": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_size_t, c_void_p]),
    "flc_weighted_sum": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int, c_float, c_void_p, c_void_p]),
    "flc_fedopt_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_double, c_double, c_double, c_void_p]),
    "flc_model_fold": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p,
                               c_int, c_double, c_double, c_double, c_void_p]),
    "flc_avg_and_gradients": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                      c_int, c_float, c_void_p]),
    "flc_model_fold_server": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                      c_int, c_float, c_double, c_void_p]),
    "flc_delta_flatten": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "flc_delta_count_nonzero_at": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p]),
    "flc_count_nonzero_at_batch": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "flc_feddr_combine": (
        c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_int, c_float, c_void_p]
    ),
    "flc_probe_set": (c_int, [c_char_p]),
    "flc_probe_read": (c_int, [POINTER(c_double), POINTER(c_int64)]),
}


class FlcError(RuntimeError):
    """A C-ABI call returned a non-zero status."""


_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load ``libflcodec.so`` (once) and attach the signatures; raise loudly if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C fl_sim_amd/csrc` (there is no CPU fallback)"
            )
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("FLC_LIB") and not hasattr(lib, name):
                continue  # (a calibration build of an older revision, A/B runs only: its missing entries stay unbound)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.flc_abi_version() != 1:
            raise ImportError(f"libflcodec ABI {lib.flc_abi_version()} != 1")
        _lib = lib
        return lib


def call(name: str, *args) -> None:
    """Call ``name`` and raise :class:`FlcError` with the library's message on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != FLC_OK:
        msg = lib.flc_last_error().decode(errors="replace")
        raise FlcError(f"{name} failed with status {rc}: {msg}")


def size(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
