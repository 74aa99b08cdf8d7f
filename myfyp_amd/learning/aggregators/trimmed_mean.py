"""Coordinate-wise trimmed mean (robust aggregation for the FYP Byzantine experiments,
``exp_SAVE3.txt:60-234``). Not in the reference; complements FedMedian."""

from __future__ import annotations

from typing import List

from myfyp_amd.learning.aggregators._math import trimmed_mean
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class TrimmedMean(Aggregator):
    """Drop the ``beta`` fraction of extreme values per coordinate, average the rest."""

    collective_kind = "trimmed_mean"

    def __init__(self, node_name: str = "unknown", beta: float = 0.1) -> None:
        super().__init__(node_name)
        self.beta = beta
        self.partial_aggregation = False

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if not models:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        params = trimmed_mean([m.get_parameters() for m in models], self.beta)
        contributors: List[str] = []
        for m in models:
            contributors += m.get_contributors()
        return models[0].build_copy(params=params, num_samples=sum(m.get_num_samples() for m in models), contributors=contributors)
