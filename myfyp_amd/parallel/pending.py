"""Deferred device results: the round's hot path never waits for the GPU.

Fit statistics and evaluation results are copied device→pinned-host asynchronously; a
:class:`Pending` stands for them until the process's :class:`Resolver` thread (shared by every engine group and device) has waited on
the copy's completion event (``hipEventSynchronize`` releases the GIL) and runs the callbacks
(metric logging). Results resolve in submission (stream) order, so a blocking ``result()`` on a
later item implies every earlier one is resolved too.
"""

from __future__ import annotations

import queue
import threading
from typing import Any, Callable, List, Optional


_STATE = threading.Lock()  # guards every Pending's state (held for a few instructions at a time)


class Pending:
    """A value produced later on the resolver thread (a tiny future).

    Cheap to create: the round driver makes a few dozen per round (one per peer and result, plus
    ``map`` chains), so there is no per-instance lock or event. State changes happen under one
    module-wide lock; a thread that blocks in :meth:`result` creates the event it waits on."""

    __slots__ = ("_done", "_value", "_exc", "_cbs", "_ev")

    def __init__(self) -> None:
        self._done = False
        self._value: Any = None
        self._exc: Optional[BaseException] = None
        self._cbs: Optional[List[Callable[[Any], None]]] = None
        self._ev: Optional[threading.Event] = None

    @classmethod
    def completed(cls, value: Any) -> "Pending":
        p = cls()
        p._value = value
        p._done = True
        return p

    def done(self) -> bool:
        return self._done

    def set_result(self, value: Any) -> None:
        with _STATE:
            self._value = value
            self._done = True
            cbs, self._cbs = self._cbs, None
            ev = self._ev
        if ev is not None:
            ev.set()
        for cb in cbs or ():
            cb(value)

    def set_exception(self, exc: BaseException) -> None:
        with _STATE:
            self._exc = exc
            self._done = True
            self._cbs = None
            ev = self._ev
        if ev is not None:
            ev.set()

    def result(self, timeout: Optional[float] = None) -> Any:
        if not self._done:
            with _STATE:
                if not self._done and self._ev is None:
                    self._ev = threading.Event()
                ev = self._ev
            if ev is not None and not ev.wait(timeout):
                raise TimeoutError("pending device result not ready")
        if self._exc is not None:
            raise self._exc
        return self._value

    def add_done_callback(self, fn: Callable[[Any], None]) -> None:
        with _STATE:
            if not self._done:
                if self._cbs is None:
                    self._cbs = []
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
        with _STATE:
            if not self._done:
                out = Pending()

                def cb(v: Any) -> None:
                    try:
                        out.set_result(fn(v))
                    except BaseException as e:  # surfaced to whoever waits on the Pending
                        out.set_exception(e)

                if self._cbs is None:
                    self._cbs = []
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
