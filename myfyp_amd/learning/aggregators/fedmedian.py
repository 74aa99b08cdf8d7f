"""Coordinate-wise median (parity target: ``p2pfl/learning/aggregators/fedmedian.py:29-65``).

The reference raises ``NotImplementedError`` before computing (``fedmedian.py:47``); this one is
implemented: per-coordinate median across the received models (Yin et al., 2018). On the collective
plane: all-gather + the ``coordinate_median`` HIP kernel (sorting network in registers).
"""

from __future__ import annotations

from typing import List

from myfyp_amd.learning.aggregators._math import coordinate_median
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class FedMedian(Aggregator):
    """Byzantine-robust coordinate median."""

    collective_kind = "median"

    def __init__(self, node_name: str = "unknown") -> None:
        super().__init__(node_name)
        self.partial_aggregation = False

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if len(models) == 0:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        params = coordinate_median([m.get_parameters() for m in models])
        contributors: List[str] = []
        for m in models:
            contributors += m.get_contributors()
        return models[0].build_copy(params=params, num_samples=sum(m.get_num_samples() for m in models), contributors=contributors)
