"""Node-aware logger with metric storage (parity: ``p2pfl/management/logger/logger.py:87-454``).

Behaviour kept from the reference:

* ``log_metric(addr, metric, value, round=None, step=None)``: ``step is None`` → global metric keyed by
  the node's current experiment round, else a local (per-step) metric (``logger.py:266-308``);
* metrics of an unregistered node (or before ``experiment_started``) are dropped silently
  (``logger.py:286-290``);
* ``get_local_logs()`` / ``get_global_logs()`` return the storage shapes unchanged.

Additions: ``log_timing`` (per-stage / per-round wall timers) and round hooks so the
benchmark and profilers can bracket rounds without patching stages.
"""

from __future__ import annotations

import datetime
import logging
import threading
from typing import Any, Callable, Dict, List, Optional, Union

from myfyp_amd.experiment import Experiment
from myfyp_amd.management.metric_storage import GlobalLogsType, GlobalMetricStorage, LocalLogsType, LocalMetricStorage
from myfyp_amd.settings import Settings
from myfyp_amd.utils.lockcheck import make_lock


class NodeNotRegistered(Exception):
    """Raised when a node is not registered."""


GRAY = "\033[90m"
RED = "\033[91m"
YELLOW = "\033[93m"
GREEN = "\033[92m"
BLUE = "\033[94m"
CYAN = "\033[96m"
RESET = "\033[0m"

_LEVEL_COLORS = {"DEBUG": BLUE, "INFO": GREEN, "WARNING": YELLOW, "ERROR": RED, "CRITICAL": RED}


class ColoredFormatter(logging.Formatter):
    """Adds colour to the level name."""

    def format(self, record: logging.LogRecord) -> str:
        record = logging.makeLogRecord(record.__dict__)
        color = _LEVEL_COLORS.get(record.levelname)
        if color:
            record.levelname = f"{color}{record.levelname}{RESET}"
        if not hasattr(record, "node"):
            record.node = "-"
        return super().format(record)


class P2PFLogger:
    """Logger that knows about nodes, experiments and metrics (not a singleton by itself)."""

    def __init__(self, nodes: Optional[Dict[str, Dict[str, Any]]] = None, disable_locks: bool = False) -> None:
        self._nodes: Dict[str, Dict[Any, Any]] = nodes if nodes else {}
        self._nodes_lock = make_lock("Logger.nodes", reentrant=True)
        self.local_metrics = LocalMetricStorage(disable_locks=disable_locks)
        self.global_metrics = GlobalMetricStorage(disable_locks=disable_locks)
        self.timings: Dict[str, Dict[str, List[float]]] = {}
        self.metric_listeners: List[Callable] = []
        self._round_hooks: List[Callable[[str, str, Optional[Experiment]], None]] = []

        self._logger = logging.getLogger("myfyp_amd")
        for h in list(self._logger.handlers):  # idempotent re-initialisation (tests)
            self._logger.removeHandler(h)
        self._logger.propagate = False
        self._logger.setLevel(logging.getLevelName(Settings.LOG_LEVEL))
        stream_handler = logging.StreamHandler()
        stream_handler.setFormatter(
            ColoredFormatter(
                f"{GRAY}[ {YELLOW}%(asctime)s {GRAY}| {CYAN}%(node)s {GRAY}| %(levelname)s{GRAY} ]:{RESET} %(message)s",
                datefmt="%Y-%m-%d %H:%M:%S",
            )
        )
        self._logger.addHandler(stream_handler)

    # ------------------------------------------------------------------ setup
    def connect_web(self, url: str, key: str) -> None:
        """Connect to the web services (only the web decorator implements it)."""

    def cleanup(self) -> None:
        for node in list(self._nodes):
            self.unregister_node(node)
        for handler in list(self._logger.handlers):
            self._logger.removeHandler(handler)

    def set_level(self, level: Union[int, str]) -> None:
        self._logger.setLevel(logging.getLevelName(level) if isinstance(level, str) else level)

    def get_level(self) -> int:
        return self._logger.getEffectiveLevel()

    def get_level_name(self, lvl: int) -> str:
        return logging.getLevelName(lvl)

    # ------------------------------------------------------------------ logging
    def info(self, node: str, message: str) -> None:
        self.log(logging.INFO, node, message)

    def debug(self, node: str, message: str) -> None:
        self.log(logging.DEBUG, node, message)

    def warning(self, node: str, message: str) -> None:
        self.log(logging.WARNING, node, message)

    def error(self, node: str, message: str) -> None:
        self.log(logging.ERROR, node, message)

    def critical(self, node: str, message: str) -> None:
        self.log(logging.CRITICAL, node, message)

    def log(self, level: int, node: str, message: str) -> None:
        if level not in (logging.DEBUG, logging.INFO, logging.WARNING, logging.ERROR, logging.CRITICAL):
            raise ValueError(f"Invalid level: {level}")
        if self._logger.isEnabledFor(level):
            self._logger.log(level, message, extra={"node": node})

    # ------------------------------------------------------------------ metrics
    def log_metric(self, addr: str, metric: str, value: float, round: Optional[int] = None, step: Optional[int] = None) -> None:
        """Log a metric; dropped if the node has not started an experiment (reference semantics).
        ``round`` overrides the experiment's current round (the reference ignores it)."""
        self.log_metric_at(addr, self.experiment_snapshot(addr), metric, value, step=step, round=round)

    def experiment_snapshot(self, addr: str) -> Optional[tuple]:
        """``(exp_name, round)`` of ``addr``'s running experiment, or None — captured when a device
        result is enqueued so a metric that lands later is filed under the round that produced it."""
        node = self._nodes.get(addr)
        experiment = node.get("Experiment") if node is not None else None
        if experiment is None or experiment.round is None or experiment.exp_name is None:
            return None
        return (experiment.exp_name, experiment.round)

    def log_metric_at(self, addr: str, snapshot: Optional[tuple], metric: str, value: float, step: Optional[int] = None, round: Optional[int] = None) -> None:
        if snapshot is None:
            return
        exp_name, rnd = snapshot
        if round is not None:
            rnd = round
        if step is None:
            self.global_metrics.add_log(exp_name, rnd, metric, addr, value)
        else:
            self.local_metrics.add_log(exp_name, rnd, metric, addr, value, step)
        for fn in list(self.metric_listeners):
            fn(addr, exp_name, rnd, metric, value, step)

    def add_metric_listener(self, fn: Callable) -> None:
        """``fn(addr, exp_name, round, metric, value, step)`` after every stored metric."""
        self.metric_listeners.append(fn)

    def remove_metric_listener(self, fn: Callable) -> None:
        if fn in self.metric_listeners:
            self.metric_listeners.remove(fn)

    def merge_logs(self, global_logs: GlobalLogsType, local_logs: LocalLogsType) -> None:
        """Insert metric records produced by another process (other ranks' peers) into this store —
        the role of the reference's central Ray logger actor (``ray_logger.py:32-250``)."""
        for exp, nodes in (global_logs or {}).items():
            for node, metrics in nodes.items():
                for metric, series in metrics.items():
                    for rnd, val in series:
                        self.global_metrics.add_log(exp, rnd, metric, node, val)
        for exp, rounds in (local_logs or {}).items():
            for rnd, nodes in rounds.items():
                for node, metrics in nodes.items():
                    for metric, series in metrics.items():
                        mine = self.local_metrics.get_all_logs().get(exp, {}).get(rnd, {}).get(node, {}).get(metric, [])
                        for step, val in series:
                            if (step, val) not in mine:
                                self.local_metrics.add_log(exp, rnd, metric, node, val, step)

    def ingest_records(self, records) -> None:
        """Store metric records ``(addr, exp, round, metric, value, step)`` produced on another rank
        (the live relay, ``management/logger/central.py``); no listener fires for them."""
        for addr, exp, rnd, metric, value, step in records:
            if step is None:
                self.global_metrics.add_log(exp, rnd, metric, addr, value)
            else:
                mine = self.local_metrics.get_all_logs().get(exp, {}).get(rnd, {}).get(addr, {}).get(metric, [])
                if (step, value) not in mine:
                    self.local_metrics.add_log(exp, rnd, metric, addr, value, step)

    def get_local_logs(self) -> LocalLogsType:
        return self.local_metrics.get_all_logs()

    def get_global_logs(self) -> GlobalLogsType:
        return self.global_metrics.get_all_logs()

    def log_timing(self, node: str, name: str, seconds: float) -> None:
        """Record a wall-clock timing (stage/fit/aggregate) for ``node``."""
        with self._nodes_lock:
            self.timings.setdefault(node, {}).setdefault(name, []).append(seconds)

    def get_timings(self) -> Dict[str, Dict[str, List[float]]]:
        return self.timings

    # ------------------------------------------------------------------ nodes
    def register_node(self, node: str, simulation: bool) -> None:
        with self._nodes_lock:
            if self._nodes.get(node) is not None:
                raise Exception(f"Node {node} already registered.")
            self._nodes[node] = {"simulation": simulation}

    def unregister_node(self, node: str) -> None:
        with self._nodes_lock:
            if node not in self._nodes:
                raise Exception(f"Node {node} not registered.")
            self._nodes.pop(node)

    def get_nodes(self) -> Dict[str, Dict[Any, Any]]:
        return self._nodes

    # ------------------------------------------------------------------ status
    def add_round_hook(self, hook: Callable[[str, str, Optional[Experiment]], None]) -> None:
        """``hook(event, node, experiment)`` with event in {experiment_started, round_started,
        round_finished, experiment_finished}."""
        self._round_hooks.append(hook)

    def remove_round_hook(self, hook: Callable) -> None:
        if hook in self._round_hooks:
            self._round_hooks.remove(hook)

    def _fire(self, event: str, node: str, experiment: Optional[Experiment]) -> None:
        for h in list(self._round_hooks):
            h(event, node, experiment)

    def experiment_started(self, node: str, experiment: Optional[Experiment]) -> None:
        with self._nodes_lock:
            if node in self._nodes:
                self._nodes[node]["Experiment"] = experiment
        self._fire("experiment_started", node, experiment)

    def experiment_finished(self, node: str) -> None:
        self._fire("experiment_finished", node, self._nodes.get(node, {}).get("Experiment"))

    def round_started(self, node: str, experiment: Optional[Experiment]) -> None:
        self._fire("round_started", node, experiment)

    def round_finished(self, node: str) -> None:
        self._fire("round_finished", node, self._nodes.get(node, {}).get("Experiment"))

    # ------------------------------------------------------------------ handlers
    def add_handler(self, handler: logging.Handler) -> None:
        self._logger.addHandler(handler)

    def log_system_metric(self, node: str, metric: str, value: float, time: datetime.datetime) -> None:
        """System metrics (CPU/RAM/GPU) are only forwarded by the web decorator."""
