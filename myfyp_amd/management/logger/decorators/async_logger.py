"""Asynchronous log emission (parity: ``decorators/async_logger.py:29-58``).

The reference uses a ``multiprocessing.Queue``; log records here never leave the process, so a
thread-side ``QueueListener`` gives the same off-the-hot-path emission without a pickling hop.
"""

from __future__ import annotations

import atexit
import logging
import queue
from logging.handlers import QueueHandler, QueueListener

from myfyp_amd.management.logger.decorators.logger_decorator import LoggerDecorator
from myfyp_amd.management.logger.logger import P2PFLogger


class AsyncLogger(LoggerDecorator):
    """Moves formatting + I/O of log records to a listener thread."""

    def __init__(self, p2pflogger: P2PFLogger) -> None:
        super().__init__(p2pflogger)
        self._queue: "queue.Queue[logging.LogRecord]" = queue.Queue(-1)
        inner = p2pflogger._logger
        self._handlers = list(inner.handlers)
        for h in self._handlers:
            inner.removeHandler(h)
        inner.addHandler(QueueHandler(self._queue))
        self._listener = QueueListener(self._queue, *self._handlers, respect_handler_level=True)
        self._listener.start()
        atexit.register(self.cleanup)

    def add_handler(self, handler: logging.Handler) -> None:
        self._listener.stop()
        self._handlers.append(handler)
        self._listener = QueueListener(self._queue, *self._handlers, respect_handler_level=True)
        self._listener.start()

    def flush(self) -> None:
        """Block until every queued record has been emitted."""
        self._listener.stop()
        self._listener = QueueListener(self._queue, *self._handlers, respect_handler_level=True)
        self._listener.start()

    def cleanup(self) -> None:
        try:
            self._listener.stop()
        except Exception:
            pass
