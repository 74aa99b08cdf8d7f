"""Process-wide logger (parity: ``p2pfl/management/logger/__init__.py:29-35``).

Assembly: ``Singleton(Web(File(Async(P2PFLogger))))`` — the Ray actor layer of the reference is
gone (one process per GPU, peers share the process logger).
"""

from myfyp_amd.management.logger.decorators.async_logger import AsyncLogger
from myfyp_amd.management.logger.decorators.file_logger import FileLogger
from myfyp_amd.management.logger.decorators.singleton_logger import SingletonLogger
from myfyp_amd.management.logger.decorators.web_logger import WebP2PFLogger
from myfyp_amd.management.logger.logger import P2PFLogger

logger = SingletonLogger(WebP2PFLogger(FileLogger(AsyncLogger(P2PFLogger(disable_locks=False)))))

__all__ = ["logger", "P2PFLogger"]
