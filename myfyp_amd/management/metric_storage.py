"""Metric storage (parity: ``p2pfl/management/metric_storage.py:24-251``).

Shapes are kept exactly because tests and the FYP harness index them:

* local:  ``{exp: {round: {node: {metric: [(step, value), ...]}}}}``
* global: ``{exp: {node: {metric: [(round, value), ...]}}}`` (first value per round kept)
"""

from __future__ import annotations

from threading import Lock
from typing import Dict, List, Optional, Tuple, Union

MetricsType = Dict[str, List[Tuple[int, float]]]
NodeLogsType = Dict[str, MetricsType]
RoundLogsType = Dict[int, NodeLogsType]
LocalLogsType = Dict[str, RoundLogsType]
GlobalLogsType = Dict[str, NodeLogsType]


class _NullLock:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class LocalMetricStorage:
    """Per-step (training) metrics for every node, round and experiment."""

    def __init__(self, disable_locks: bool = False) -> None:
        self.exp_dicts: LocalLogsType = {}
        self.lock: Optional[Lock] = None if disable_locks else Lock()

    def add_log(self, exp_name: str, round: int, metric: str, node: str, val: Union[int, float], step: int) -> None:
        with self.lock or _NullLock():
            node_logs = self.exp_dicts.setdefault(exp_name, {}).setdefault(round, {}).setdefault(node, {})
            node_logs.setdefault(metric, []).append((step, val))

    def get_all_logs(self) -> LocalLogsType:
        return self.exp_dicts

    def get_experiment_logs(self, exp: str) -> RoundLogsType:
        return self.exp_dicts[exp]

    def get_experiment_round_logs(self, exp: str, round: int) -> NodeLogsType:
        return self.exp_dicts[exp][round]

    def get_experiment_round_node_logs(self, exp: str, round: int, node: str) -> MetricsType:
        return self.exp_dicts[exp][round][node]


class GlobalMetricStorage:
    """Per-round (evaluation) metrics; only the first value logged for a round is kept."""

    def __init__(self, disable_locks: bool = False) -> None:
        self.exp_dicts: GlobalLogsType = {}
        self.lock: Optional[Lock] = None if disable_locks else Lock()
        self._seen: dict = {}  # (exp, node, metric) -> rounds already stored (O(1) first-value-wins)

    def add_log(self, exp_name: str, round: int, metric: str, node: str, val: Union[int, float]) -> None:
        with self.lock or _NullLock():
            series = self.exp_dicts.setdefault(exp_name, {}).setdefault(node, {}).setdefault(metric, [])
            seen = self._seen.get((exp_name, node, metric))
            if seen is None or len(seen) != len(series):  # (re)build if the series was edited directly
                seen = self._seen[(exp_name, node, metric)] = {r for r, _ in series}
            if round not in seen:
                seen.add(round)
                series.append((round, val))

    def get_all_logs(self) -> GlobalLogsType:
        return self.exp_dicts

    def get_experiment_logs(self, exp: str) -> NodeLogsType:
        return self.exp_dicts[exp]

    def get_experiment_node_logs(self, exp: str, node: str) -> MetricsType:
        return self.exp_dicts[exp][node]
