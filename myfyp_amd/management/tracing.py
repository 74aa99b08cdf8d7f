"""roctx ranges for timeline profiling.

The reference has no tracing spans (only ``StageWokflow.history`` and an optional yappi profile of
the MNIST example). Here the host control plane can annotate the GPU timeline: with
``Settings.TRACE_MARKERS = True`` (or ``MYFYP_ROCTX=1``), :func:`trace_range` pushes/pops roctx
ranges — every workflow stage, ``fit``, ``evaluate``, the aggregation collectives, model encode —
which ``rocprofv3 --marker-trace`` records next to the kernels they launched. The ranges are
nested per thread (roctx keeps one stack per thread), so each peer's learning thread forms its own
track. Off (default), :func:`trace_range` is a shared no-op context manager.

roctx is a host library (``librocprofiler-sdk-roctx``, falling back to the legacy ``libroctx64``);
without a profiler attached its calls return immediately, and when neither library can be loaded
tracing silently stays off.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import threading
from typing import Iterator, Optional

_LIB: Optional[ctypes.CDLL] = None
_TRIED = False
_LOCK = threading.Lock()
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


def _load() -> Optional[ctypes.CDLL]:
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    with _LOCK:
        if not _TRIED:
            rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
            for name in _CANDIDATES:
                for path in (os.path.join(rocm, "lib", name), name):
                    try:
                        lib = ctypes.CDLL(path)
                    except OSError:
                        continue
                    try:
                        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                        lib.roctxRangePushA.restype = ctypes.c_int
                        lib.roctxRangePop.argtypes = []
                        lib.roctxRangePop.restype = ctypes.c_int
                        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                        lib.roctxMarkA.restype = None
                    except AttributeError:
                        continue
                    _LIB = lib
                    break
                if _LIB is not None:
                    break
            _TRIED = True
    return _LIB


def enabled() -> bool:
    if os.environ.get("MYFYP_ROCTX", "") not in ("", "0"):
        return _load() is not None
    from myfyp_amd.settings import Settings

    return bool(Settings.TRACE_MARKERS) and _load() is not None


_NULL = contextlib.nullcontext()
_TLS = threading.local()


def depth() -> int:
    """Open ranges of the calling thread (what this module pushed)."""
    return getattr(_TLS, "depth", 0)


@contextlib.contextmanager
def _range(name: str) -> Iterator[None]:
    lib = _LIB
    lib.roctxRangePushA(name.encode())
    _TLS.depth = depth() + 1
    try:
        yield
    finally:
        _TLS.depth = depth() - 1
        lib.roctxRangePop()


def trace_range(name: str):
    """``with trace_range("fit/peer-3"):`` — a roctx range when tracing is on, else a no-op."""
    if not enabled():
        return _NULL
    return _range(name)


def traced(label: str):
    """Method/function decorator: the call runs inside ``trace_range(label[/addr])`` (``addr`` =
    the bound object's ``_self_addr`` when it has one)."""

    def deco(fn):
        import functools

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if not enabled():
                return fn(*args, **kwargs)
            addr = getattr(args[0], "_self_addr", None) if args else None
            with _range(f"{label}/{addr}" if addr else label):
                return fn(*args, **kwargs)

        return wrapper

    return deco


def mark(name: str) -> None:
    """An instantaneous roctx marker (no-op when tracing is off)."""
    if enabled():
        _LIB.roctxMarkA(name.encode())
