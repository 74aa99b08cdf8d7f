"""Loader for the in-tree native library ``myfyp_amd/_native/libmyfyp_hip.so``.

The library is plain C ABI (HIP kernels + the C++ runtime: grouped MLP engine, hipGraph capture),
called through ``ctypes`` with raw device pointers and the caller's HIP stream — no PyTorch C++
ABI coupling, no hipify. ``build()`` in ``__graft_entry__.py`` / ``python -m myfyp_amd.ops.build``
compiles it for gfx950.

Policy: on a machine with a GPU the native library is REQUIRED for device tensors (ops raise if it
is missing — a silent eager fallback would hide a broken build); on CPU-only hosts the PyTorch
reference implementations in :mod:`myfyp_amd.ops` run instead.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_LIB: Optional[ctypes.CDLL] = None
_FAST: Optional[ctypes.PyDLL] = None
_LOCK = threading.Lock()
_ERR: Optional[str] = None

LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native")
LIB_PATH = os.environ.get("MYFYP_NATIVE_LIB") or os.path.join(LIB_DIR, "libmyfyp_hip.so")  # override: diagnostics builds

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float

# name -> (restype, argtypes)
_SIGNATURES = {
    "myfyp_version": (c_int, []),
    "myfyp_last_error": (ctypes.c_char_p, []),
    # aggregation
    "myfyp_weighted_sum": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    "myfyp_stacked_weighted_sum": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_float, c_void_p]),
    "myfyp_broadcast_rows": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_coordinate_median": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    "myfyp_coordinate_median_multi": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int64, c_void_p]),
    "myfyp_scaffold_reduce": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    "myfyp_scaffold_apply": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_float, c_int64, c_void_p]),
    # optimizers over flat buffers
    "myfyp_adam_step": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p],
    ),
    "myfyp_sgd_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p]),
    # attacks / elementwise
    "myfyp_scale_add_noise": (c_int, [c_void_p, c_int64, c_float, c_float, ctypes.c_uint64, c_void_p]),

    # grouped MLP engine
    "mlp_shape_ok": (c_int, [c_int, c_int, c_int, c_int]),
    "mlp_engine_create": (c_void_p, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "mlp_engine_destroy": (None, [c_void_p]),
    "mlp_engine_numel": (c_int64, [c_void_p]),
    "mlp_engine_bind_params": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64]),
    "mlp_engine_set_train_data": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int]),
    "mlp_engine_set_test_data": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "mlp_engine_set_counts": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mlp_engine_set_optimizer": (c_int, [c_void_p, c_int, c_float, c_float, c_float, c_float, c_float, c_float, c_int, c_float]),
    "mlp_engine_set_extras": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlp_engine_begin": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mlp_engine_run_epoch": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mlp_engine_run_epoch_pub": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "mlp_engine_set_train_x16": (c_int, [c_void_p, c_void_p]),
    "mlp_engine_drain_prep": (c_int, [c_void_p]),
    "mlp_engine_x_direct": (c_int, [c_void_p]),
    "mlp_engine_x_direct_build": (c_int, []),
    "mlp_engine_run_epoch_eager": (c_int, [c_void_p, c_void_p, c_void_p]),
    "mlp_engine_read_stats": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlp_engine_eval": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mlp_engine_stats_async": (c_int, [c_void_p, c_int, c_void_p]),
    "mlp_engine_eval_async": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "mlp_engine_fetch": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "mlp_engine_ring_size": (c_int, []),
    "mlp_engine_set_persistent": (c_int, [c_void_p, c_int]),
    "mlp_engine_zero_state": (c_int, [c_void_p, c_void_p]),
    "mlp_engine_set_shuffle": (c_int, [c_void_p, c_int]),
    "mlp_engine_set_epoch_seed": (c_int, [c_void_p, ctypes.c_uint64]),
    "mlp_engine_set_next_epoch_seed": (c_int, [c_void_p, ctypes.c_uint64]),
    "myfyp_fedavg_stacked_reduce": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_fedavg_stacked_apply": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_fedavg_stacked_local": (c_int, [c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "myfyp_fedavg_bucket_reduce": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_fedavg_bucket_apply": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_fedavg_bucket_reduce2": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_fedavg_delayed_land": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "myfyp_neighbor_mix_stacked": (c_int, [c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "mlp_engine_uses_persistent": (c_int, [c_void_p]),
    "mlp_engine_set_precision": (c_int, [c_void_p, c_int]),
    "mlp_f32_ok": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "mlp_engine_set_w2chk": (c_int, [c_void_p, c_void_p]),
    "mlp_engine_recoveries": (c_int, [c_void_p]),
    "mlp_engine_graph_launch_stats": (c_int, [c_void_p, c_void_p]),
    "mlp_engine_set_f32_ks": (c_int, [c_void_p, c_int]),
    "mlp_engine_set_reserved_cus": (c_int, [c_void_p, c_int]),
    "mlp_engine_f32_ks": (c_int, [c_void_p]),
    "mlp_engine_set_f32_variant": (c_int, [c_void_p, c_int]),
    "mlp_engine_f32_variant": (c_int, [c_void_p]),
    "mlp_engine_debug_giveup": (c_int, [c_void_p, c_int, c_int]),
    "mlp_engine_debug_poison_flags": (c_int, [c_void_p, c_int]),
    "mlp_engine_prepare": (c_int, [c_void_p, c_void_p]),
    "myfyp_warm_all": (c_int, [c_int]),
    "mlp_set_plain_pub": (c_int, [c_int]),  # single-XCD hand-off mode override (-1: MYFYP_F32_PLAIN_PUB)
    "mlp_debug_plain_seen": (c_int, [c_void_p]),
    "mlp_debug_stamps": (c_int, [c_void_p]),  # only in the -DMLP_STAMPS diagnostics build
    "mlp_debug_persistent_f32_stamps": (c_int, [c_void_p]),  # likewise
}


def load(required: bool = False) -> Optional[ctypes.CDLL]:
    """Return the native library (loading it once). ``required`` raises if unavailable."""
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None and _ERR is None:
            if not os.path.exists(LIB_PATH):
                _ERR = f"native library not built: {LIB_PATH} (run python -m myfyp_amd.ops.build)"
            else:
                try:
                    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                    for name, (res, args) in _SIGNATURES.items():
                        fn = getattr(lib, name, None)
                        if fn is None:
                            continue
                        fn.restype = res
                        fn.argtypes = args
                    _LIB = lib
                except OSError as e:
                    _ERR = f"failed to load {LIB_PATH}: {e}"
    if _LIB is None and required:
        raise RuntimeError(_ERR or "native library unavailable")
    return _LIB


def load_fast() -> ctypes.PyDLL:
    """The same library bound as a ``PyDLL``: calls keep the GIL. Use it ONLY for entry points that
    merely enqueue work (launches, async copies, parameter setters). Releasing and re-taking the GIL
    around a microsecond-long call costs far more than the call when several peer threads run
    Python concurrently: the caller queues behind whichever thread got the GIL (up to the
    interpreter's switch interval); blocking calls (event waits) go through :func:`load`."""
    global _FAST
    if _FAST is not None:
        return _FAST
    load(required=True)
    with _LOCK:
        if _FAST is None:
            lib = ctypes.PyDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(lib, name, None)
                if fn is None:
                    continue
                fn.restype = res
                fn.argtypes = args
            _FAST = lib
    return _FAST


def debug_update_scale() -> float:
    """Mutation-testing knob (``MYFYP_DEBUG_LR_SCALE``, default 1): the fused engines multiply their
    learning rate by it, so every update they apply is off by that factor while the torch references
    the tests compare against are not. Used once to show which tests catch a 5 % update error
    (``profiles/r5_mutation``); never set in normal runs."""
    v = os.environ.get("MYFYP_DEBUG_LR_SCALE")
    return float(v) if v else 1.0


_WARM: set = set()


def warm_device(index: int, family: str = "mlp") -> None:
    """Load the kernel units an engine ``family`` ("mlp" or "cnn") launches on device ``index`` (the
    current device), once per process, device and family: engine prewarm. A unit's first launch
    would otherwise load it then, waiting for the kernels in flight (``myfyp_warm_all``)."""
    key = (index, family)
    if key in _WARM:
        return
    lib = load(required=True)
    fn = getattr(lib, "myfyp_warm_all", None)
    if fn is not None:
        bad = int(fn(1 if family == "mlp" else 2))
        if bad:
            raise RuntimeError(f"native code objects: {bad} kernel unit(s) failed to load on device {index}")
    _WARM.add(key)


def available() -> bool:
    return load() is not None


def error() -> Optional[str]:
    load()
    return _ERR


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _LIB.myfyp_last_error().decode() if _LIB is not None else "?"
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")
