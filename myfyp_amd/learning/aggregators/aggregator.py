"""Stateful round aggregator (parity: ``p2pfl/learning/aggregators/aggregator.py:35-270``).

Semantics kept: ``set_nodes_to_aggregate`` (refused while a round runs), ``add_model`` accepts
contributions whose contributors ⊆ train set and are disjoint from what is already held, the finish
event fires when every train-set node contributed, ``wait_and_get_aggregation`` aggregates whatever
arrived (partial on timeout), ``get_model(except_nodes)`` returns a partial aggregate (when
supported) or one remaining model.

Fix: the reference releases an un-held lock on the empty-contributors path.

Collective data plane: an aggregator also exposes ``collective_kind`` which tells the RCCL weights
plane which reduction implements it (``"mean"`` → one weighted all-reduce, ``"median"`` →
all-gather + per-coordinate median kernel, ``None`` → host fallback).
"""

from __future__ import annotations

import threading
from typing import List, Optional

from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.utils.lockcheck import make_lock


class NoModelsToAggregateError(Exception):
    """There is nothing to aggregate."""


class Aggregator:
    """Collects the train set's models for one round and reduces them."""

    #: how the collective (RCCL) weights plane implements this aggregator
    collective_kind: Optional[str] = None

    def __init__(self, node_name: str = "unknown") -> None:
        self.node_name = node_name
        self._train_set: List[str] = []
        self._models: List[P2PFLModel] = []
        self.partial_aggregation = False
        self._agg_lock = make_lock("Aggregator.agg")
        self._finish_aggregation_event = threading.Event()
        self._finish_aggregation_event.set()

    # ------------------------------------------------------------------ to implement
    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        raise NotImplementedError

    def get_required_callbacks(self) -> List[str]:
        return []

    # ------------------------------------------------------------------ round state
    def set_node_name(self, name: str) -> None:
        self.node_name = name

    def set_nodes_to_aggregate(self, nodes_to_aggregate: List[str]) -> None:
        if not self._finish_aggregation_event.is_set():
            raise Exception("It is not possible to set nodes to aggregate when the aggregation is running.")
        self._train_set = list(nodes_to_aggregate)
        self._finish_aggregation_event.clear()

    def clear(self) -> None:
        with self._agg_lock:
            self._train_set = []
            self._models = []
            self._finish_aggregation_event.set()

    def get_aggregated_models(self) -> List[str]:
        out: List[str] = []
        for m in self._models:
            out += m.get_contributors()
        return out

    def add_model(self, model: P2PFLModel) -> List[str]:
        contributors = model.contributors
        if not contributors:
            logger.debug(self.node_name, "Received a model without a list of contributors.")
            return []
        with self._agg_lock:
            aggregated = self.get_aggregated_models()
            if len(self._train_set) <= len(aggregated):
                logger.debug(self.node_name, "🚫 Received a model when is not needed (already aggregated).")
                return []
            if not all(n in self._train_set for n in contributors):
                logger.debug(self.node_name, f"Can't add a model from a node ({contributors}) that is not in the training set.")
                return []
            if any(n in aggregated for n in contributors):
                logger.debug(self.node_name, f"Can't add a model from a node ({contributors}) that is already aggregated.")
                return []
            self._models.append(model)
            aggregated = self.get_aggregated_models()
            logger.info(self.node_name, f"🧩 Model added ({len(aggregated)}/{len(self._train_set)}) from {contributors}")
            if len(aggregated) >= len(self._train_set):
                self._finish_aggregation_event.set()
            return aggregated

    def wait_and_get_aggregation(self, timeout: Optional[float] = None) -> P2PFLModel:
        if timeout is None:
            timeout = Settings.AGGREGATION_TIMEOUT
        event_set = self._finish_aggregation_event.wait(timeout=timeout)
        missing = self.get_missing_models()
        if not event_set:
            logger.info(self.node_name, f"⏳ Aggregation wait timed out. Missing models: {missing}")
        elif missing:
            logger.info(self.node_name, f"❌ Aggregation event set, but missing models:  {missing}")
        else:
            logger.info(self.node_name, "🧠 Aggregating models.")
        with self._agg_lock:
            models = list(self._models)
        return self.aggregate(models)

    def get_missing_models(self) -> set:
        return set(self._train_set) - set(self.get_aggregated_models())

    def get_model(self, except_nodes: List[str]) -> P2PFLModel:
        with self._agg_lock:
            models = list(self._models)
        candidates = [m for m in models if all(n not in except_nodes for n in m.get_contributors())]
        if self.partial_aggregation:
            return self.aggregate(candidates)
        if not candidates:
            raise NoModelsToAggregateError("No remaining models available for aggregation.")
        return candidates[0]
