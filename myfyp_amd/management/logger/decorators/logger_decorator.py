"""Pure-delegation logger decorator (parity: ``decorators/logger_decorator.py:30-243``)."""

from __future__ import annotations

import datetime
import logging
from typing import Any, Callable, Dict, Optional, Union

from myfyp_amd.experiment import Experiment
from myfyp_amd.management.logger.logger import P2PFLogger
from myfyp_amd.management.metric_storage import GlobalLogsType, LocalLogsType


class LoggerDecorator(P2PFLogger):
    """Forwards every call to the wrapped logger."""

    def __init__(self, logger: P2PFLogger) -> None:  # noqa: D107 - no super() on purpose
        self._p2pflogger = logger

    def __getattr__(self, name: str) -> Any:
        return getattr(self._p2pflogger, name)

    def connect_web(self, url: str, key: str) -> None:
        self._p2pflogger.connect_web(url, key)

    def cleanup(self) -> None:
        self._p2pflogger.cleanup()

    def set_level(self, level: Union[int, str]) -> None:
        self._p2pflogger.set_level(level)

    def get_level(self) -> int:
        return self._p2pflogger.get_level()

    def get_level_name(self, lvl: int) -> str:
        return self._p2pflogger.get_level_name(lvl)

    def log(self, level: int, node: str, message: str) -> None:
        self._p2pflogger.log(level, node, message)

    def log_metric(self, addr: str, metric: str, value: float, round: Optional[int] = None, step: Optional[int] = None) -> None:
        self._p2pflogger.log_metric(addr, metric, value, round, step)

    def get_local_logs(self) -> LocalLogsType:
        return self._p2pflogger.get_local_logs()

    def ingest_records(self, records) -> None:
        self._p2pflogger.ingest_records(records)

    def get_global_logs(self) -> GlobalLogsType:
        return self._p2pflogger.get_global_logs()

    def log_timing(self, node: str, name: str, seconds: float) -> None:
        self._p2pflogger.log_timing(node, name, seconds)

    def get_timings(self):
        return self._p2pflogger.get_timings()

    def register_node(self, node: str, simulation: bool) -> None:
        self._p2pflogger.register_node(node, simulation)

    def unregister_node(self, node: str) -> None:
        self._p2pflogger.unregister_node(node)

    def get_nodes(self) -> Dict[str, Dict[Any, Any]]:
        return self._p2pflogger.get_nodes()

    def add_round_hook(self, hook: Callable) -> None:
        self._p2pflogger.add_round_hook(hook)

    def remove_round_hook(self, hook: Callable) -> None:
        self._p2pflogger.remove_round_hook(hook)

    def experiment_started(self, node: str, experiment: Optional[Experiment]) -> None:
        self._p2pflogger.experiment_started(node, experiment)

    def experiment_finished(self, node: str) -> None:
        self._p2pflogger.experiment_finished(node)

    def round_started(self, node: str, experiment: Optional[Experiment]) -> None:
        self._p2pflogger.round_started(node, experiment)

    def round_finished(self, node: str) -> None:
        self._p2pflogger.round_finished(node)

    def add_handler(self, handler: logging.Handler) -> None:
        self._p2pflogger.add_handler(handler)

    def log_system_metric(self, node: str, metric: str, value: float, time: datetime.datetime) -> None:
        self._p2pflogger.log_system_metric(node, metric, value, time)
