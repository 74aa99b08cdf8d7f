"""Web dashboard sink (parity: ``decorators/web_logger.py:36-196``)."""

from __future__ import annotations

import datetime
import logging
from typing import Dict, Optional

from myfyp_amd.management.logger.decorators.logger_decorator import LoggerDecorator
from myfyp_amd.management.logger.logger import P2PFLogger
from myfyp_amd.management.node_monitor import NodeMonitor
from myfyp_amd.management.web_services import P2pflWebServices


class DictFormatter(logging.Formatter):
    """Log record → the dashboard's log dict (``timestamp``, ``node``, ``level``, ``message``)."""

    def format(self, record: logging.LogRecord) -> dict:  # type: ignore[override]
        return {
            "timestamp": datetime.datetime.fromtimestamp(record.created),
            "node": getattr(record, "node", "-"),
            "level": record.levelno,
            "message": record.getMessage(),
        }


class P2pflWebLogHandler(logging.Handler):
    """Forwards log records to the dashboard."""

    def __init__(self, p2pfl_web: P2pflWebServices) -> None:
        super().__init__()
        self._p2pfl_web = p2pfl_web
        self.setFormatter(DictFormatter())

    def emit(self, record: logging.LogRecord) -> None:
        try:
            d = self.formatter.format(record)  # type: ignore[union-attr]
            self._p2pfl_web.send_log(d["timestamp"], d["node"], d["level"], d["message"])
        except Exception:
            pass


class WebP2PFLogger(LoggerDecorator):
    """Adds the REST sink and a per-node ``NodeMonitor`` once ``connect_web`` is called."""

    def __init__(self, p2pflogger: P2PFLogger) -> None:
        super().__init__(p2pflogger)
        self._p2pfl_web_services: Optional[P2pflWebServices] = None
        self._monitors: Dict[str, NodeMonitor] = {}

    def connect_web(self, url: str, key: str) -> None:
        self._p2pfl_web_services = P2pflWebServices(url, key)
        self._p2pflogger.add_handler(P2pflWebLogHandler(self._p2pfl_web_services))

    def log_metric(self, addr: str, metric: str, value: float, round: Optional[int] = None, step: Optional[int] = None) -> None:
        super().log_metric(addr, metric, value, round, step)
        if self._p2pfl_web_services is None:
            return
        exp = self.get_nodes().get(addr, {}).get("Experiment")
        if exp is None:
            return
        try:
            if step is None:
                self._p2pfl_web_services.send_global_metric(exp.exp_name, exp.round, metric, addr, value)
            else:
                self._p2pfl_web_services.send_local_metric(exp.exp_name, exp.round, metric, addr, value, step)
        except Exception:
            pass

    def log_system_metric(self, node: str, metric: str, value: float, time: datetime.datetime) -> None:
        if self._p2pfl_web_services is not None:
            try:
                self._p2pfl_web_services.send_system_metric(node, metric, value, time)
            except Exception:
                pass

    def register_node(self, node: str, simulation: bool) -> None:
        super().register_node(node, simulation)
        if self._p2pfl_web_services is not None:
            try:
                self._p2pfl_web_services.register_node(node, simulation)
            except Exception:
                pass
            mon = NodeMonitor(node, self.log_system_metric)
            self._monitors[node] = mon
            mon.start()

    def unregister_node(self, node: str) -> None:
        super().unregister_node(node)
        mon = self._monitors.pop(node, None)
        if mon is not None:
            mon.stop()
        if self._p2pfl_web_services is not None:
            try:
                self._p2pfl_web_services.unregister_node(node)
            except Exception:
                pass
