"""Lock-order checking for the host control plane.

The reference coordinates its threads (learning thread, gossiper, heartbeater, server pool, command
handlers) with ad-hoc locks and has no lock-order checking (``node_state.py:74-80``,
``aggregator.py:52-54``, ``gossiper.py:61-65``, ``neighbors.py:40``, ``metric_storage.py:53``). Here
the framework's mutexes are created through :func:`make_lock`. With checking off (default) that is
a plain ``threading.Lock``/``RLock`` — zero overhead. With ``MYFYP_LOCK_CHECK=1`` in the
environment or ``Settings.LOCK_CHECK`` set before the objects are built, every lock is a
:class:`CheckedLock` that records, per thread, which named locks are held when another is taken.
The first time an acquisition closes a cycle in that "held-before" graph (A taken under B somewhere,
B taken under A elsewhere — a potential deadlock even if the schedule never hit it) the inversion is
recorded with both call sites; ``LOCK_CHECK = "raise"`` turns it into :class:`LockOrderError`.

Locks of one name are one node of the graph (two NodeStates' vote locks are the same class of lock);
nesting two instances of the same name is not reported.
"""

from __future__ import annotations

import os
import threading
import traceback
from typing import Dict, List, Optional, Tuple

_ENV = os.environ.get("MYFYP_LOCK_CHECK", "").strip().lower()


class LockOrderError(RuntimeError):
    """Two named locks were taken in opposite orders (potential deadlock)."""


def _mode() -> str:
    if _ENV not in ("", "0", "false", "off"):
        return "raise" if _ENV == "raise" else "record"
    from myfyp_amd.settings import Settings

    v = getattr(Settings, "LOCK_CHECK", False)
    if v in (False, None, 0, "", "0", "off"):
        return ""
    return "raise" if v == "raise" else "record"


def enabled() -> bool:
    return _mode() != ""


class _Graph:
    def __init__(self) -> None:
        self.lock = threading.Lock()
        self.edges: Dict[str, Dict[str, str]] = {}  # held -> {acquired: first call site}
        self.violations: List[Tuple[str, str, str, str]] = []  # (held, acquiring, site, reverse site)
        self._reported: set = set()

    def _path(self, src: str, dst: str) -> Optional[List[str]]:
        stack, seen = [(src, [src])], {src}
        while stack:
            node, path = stack.pop()
            if node == dst:
                return path
            for nxt in self.edges.get(node, ()):
                if nxt not in seen:
                    seen.add(nxt)
                    stack.append((nxt, path + [nxt]))
        return None

    def note(self, held: List["CheckedLock"], acquiring: "CheckedLock") -> Optional[str]:
        names = [h.name for h in held if h.name != acquiring.name]
        if not names:
            return None
        site = None
        msg = None
        with self.lock:
            for h in names:
                out = self.edges.setdefault(h, {})
                if acquiring.name in out:
                    continue
                site = site or "".join(traceback.format_stack(limit=6)[:-2])
                back = self._path(acquiring.name, h)
                out[acquiring.name] = site
                if back is not None and (h, acquiring.name) not in self._reported:
                    self._reported.add((h, acquiring.name))
                    rsite = self.edges[back[0]].get(back[1], "?") if len(back) > 1 else "?"
                    self.violations.append((h, acquiring.name, site, rsite))
                    msg = f"lock-order inversion: {acquiring.name!r} taken while holding {h!r}, but elsewhere {' -> '.join(back)}"
        return msg


_GRAPH = _Graph()
_TLS = threading.local()


def _held() -> List["CheckedLock"]:
    h = getattr(_TLS, "held", None)
    if h is None:
        h = _TLS.held = []
    return h


class CheckedLock:
    """Named (R)Lock that feeds the held-before graph."""

    def __init__(self, name: str, reentrant: bool = False) -> None:
        self.name = name
        self.reentrant = reentrant
        self._lock = threading.RLock() if reentrant else threading.Lock()
        self._owner: Optional[int] = None
        self._depth = 0

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        me = threading.get_ident()
        if not (self.reentrant and self._owner == me):
            msg = _GRAPH.note(_held(), self)
            if msg is not None:
                from myfyp_amd.management.logger import logger

                logger.warning("lockcheck", msg)
                if _mode() == "raise":
                    raise LockOrderError(msg)
        ok = self._lock.acquire(blocking, timeout)
        if ok:
            if self._owner == me:
                self._depth += 1
            else:
                self._owner, self._depth = me, 1
                _held().append(self)
        return ok

    def release(self) -> None:
        if self._owner == threading.get_ident():
            self._depth -= 1
            if self._depth == 0:
                self._owner = None
                held = _held()
                for i in range(len(held) - 1, -1, -1):
                    if held[i] is self:
                        del held[i]
                        break
        self._lock.release()

    def locked(self) -> bool:
        return self._owner is not None

    def __enter__(self) -> "CheckedLock":
        self.acquire()
        return self

    def __exit__(self, *exc) -> None:
        self.release()


def make_lock(name: str, reentrant: bool = False):
    """A mutex for the framework's shared state: plain when checking is off, checked otherwise."""
    if enabled():
        return CheckedLock(name, reentrant)
    return threading.RLock() if reentrant else threading.Lock()


def violations() -> List[Tuple[str, str, str, str]]:
    with _GRAPH.lock:
        return list(_GRAPH.violations)


def lock_graph() -> Dict[str, List[str]]:
    with _GRAPH.lock:
        return {k: sorted(v) for k, v in _GRAPH.edges.items()}


def reset() -> None:
    with _GRAPH.lock:
        _GRAPH.edges.clear()
        _GRAPH.violations.clear()
        _GRAPH._reported.clear()
