"""Deferred device results: the round's hot path never waits for the GPU.

Fit statistics and evaluation results are copied device→pinned-host asynchronously; a
:class:`Pending` stands for them until one :class:`Resolver` thread per engine group has waited on
the copy's completion event (``hipEventSynchronize`` releases the GIL) and runs the callbacks
(metric logging). Results resolve in submission (stream) order, so a blocking ``result()`` on a
later item implies every earlier one is resolved too.
"""

from __future__ import annotations

import queue
import threading
from typing import Any, Callable, List, Optional


class Pending:
    """A value produced later on the resolver thread (a tiny future)."""

    __slots__ = ("_ev", "_value", "_exc", "_cbs", "_lock")

    def __init__(self) -> None:
        self._ev = threading.Event()
        self._value: Any = None
        self._exc: Optional[BaseException] = None
        self._cbs: List[Callable[[Any], None]] = []
        self._lock = threading.Lock()

    @classmethod
    def completed(cls, value: Any) -> "Pending":
        p = cls()
        p.set_result(value)
        return p

    def done(self) -> bool:
        return self._ev.is_set()

    def set_result(self, value: Any) -> None:
        with self._lock:
            self._value = value
            self._ev.set()
            cbs, self._cbs = self._cbs, []
        for cb in cbs:
            cb(value)

    def set_exception(self, exc: BaseException) -> None:
        with self._lock:
            self._exc = exc
            self._ev.set()
            self._cbs = []

    def result(self, timeout: Optional[float] = None) -> Any:
        if not self._ev.wait(timeout):
            raise TimeoutError("pending device result not ready")
        if self._exc is not None:
            raise self._exc
        return self._value

    def add_done_callback(self, fn: Callable[[Any], None]) -> None:
        with self._lock:
            if not self._ev.is_set():
                self._cbs.append(fn)
                return
        if self._exc is None:
            fn(self._value)

    def map(self, fn: Callable[[Any], Any]) -> "Pending":
        out = Pending()
        self.add_done_callback(lambda v: out.set_result(fn(v)))
        return out

    def map_off_thread(self, fn: Callable[[Any], Any]) -> "Pending":
        """Like :meth:`map`, but ``fn`` never runs on the calling thread: if the value is already
        there, ``fn`` goes to the shared resolver thread (FIFO behind earlier results). For heavy
        callbacks (metric logging) issued from the round driver: after a device synchronisation
        every result of the queued rounds is already resolved, and running their logging inline
        held the next launch back by 0.7 ms (``profiles/r5_start``)."""
        with self._lock:
            if not self._ev.is_set():
                out = Pending()

                def cb(v: Any) -> None:
                    try:
                        out.set_result(fn(v))
                    except BaseException as e:  # surfaced to whoever waits on the Pending
                        out.set_exception(e)

                self._cbs.append(cb)
                return out
        if self._exc is not None:
            out = Pending()
            out.set_exception(self._exc)
            return out
        v = self._value
        return Resolver.shared().submit(lambda: fn(v))


def resolve(value: Any) -> Any:
    """Value of ``value`` (waiting if it is a :class:`Pending`)."""
    return value.result() if isinstance(value, Pending) else value


class Resolver:
    """FIFO worker that runs ``fetch()`` (blocking on a device event) and completes a Pending."""

    _shared: Optional["Resolver"] = None
    _shared_lock = threading.Lock()

    def __init__(self, name: str) -> None:
        self._q: "queue.Queue" = queue.Queue()
        self._thread = threading.Thread(target=self._loop, name=name, daemon=True)
        self._thread.start()

    @classmethod
    def shared(cls) -> "Resolver":
        """The process-wide resolver (FIFO over every engine group's results)."""
        with cls._shared_lock:
            if cls._shared is None:
                cls._shared = cls("device-results")
            return cls._shared

    def submit(self, fetch: Callable[[], Any]) -> Pending:
        p = Pending()
        self._q.put((fetch, p))
        return p

    def flush(self) -> None:
        self._q.join()

    def _loop(self) -> None:
        while True:
            fetch, p = self._q.get()
            try:
                p.set_result(fetch())
            except BaseException as e:  # surfaced to whoever waits on the Pending
                p.set_exception(e)
            finally:
                self._q.task_done()
