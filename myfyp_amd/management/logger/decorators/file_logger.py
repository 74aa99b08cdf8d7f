"""Rotating file log sink (parity: ``decorators/file_logger.py:30-53``)."""

from __future__ import annotations

import logging
import os
from logging.handlers import RotatingFileHandler

from myfyp_amd.management.logger.decorators.logger_decorator import LoggerDecorator
from myfyp_amd.management.logger.logger import P2PFLogger
from myfyp_amd.settings import Settings


class FileLogger(LoggerDecorator):
    """Adds a ``RotatingFileHandler(LOG_DIR/p2pfl.log, 1 MB x 3)`` lazily on first use."""

    def __init__(self, p2pflogger: P2PFLogger) -> None:
        super().__init__(p2pflogger)
        self._file_handler_ready = False

    def setup_file_handler(self) -> None:
        if self._file_handler_ready:
            return
        os.makedirs(Settings.LOG_DIR, exist_ok=True)
        handler = RotatingFileHandler(os.path.join(Settings.LOG_DIR, "p2pfl.log"), maxBytes=1_000_000, backupCount=3)
        handler.setFormatter(logging.Formatter("[ %(asctime)s | %(node)s | %(levelname)s ]: %(message)s"))
        self._p2pflogger.add_handler(handler)
        self._file_handler_ready = True
