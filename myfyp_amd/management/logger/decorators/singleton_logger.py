"""Singleton logger (parity: ``decorators/singleton_logger.py:24-27``)."""

from myfyp_amd.management.logger.decorators.logger_decorator import LoggerDecorator
from myfyp_amd.utils.singleton import SingletonMeta


class SingletonLogger(LoggerDecorator, metaclass=SingletonMeta):
    """Process-wide logger instance."""
