"""Federated Averaging (parity: ``p2pfl/learning/aggregators/fedavg.py:29-77``).

Sample-weighted mean; supports partial aggregation. On the collective plane it is one weighted
all-reduce (``collective_kind = "mean"``); for device-resident models the reduction is the fused
``weighted_average`` HIP kernel.
"""

from __future__ import annotations

from typing import List

from myfyp_amd.learning.aggregators._math import weighted_mean
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class FedAvg(Aggregator):
    """McMahan et al., 2016 — https://arxiv.org/abs/1602.05629."""

    collective_kind = "mean"

    def __init__(self, node_name: str = "unknown") -> None:
        super().__init__(node_name)
        self.partial_aggregation = True

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if len(models) == 0:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        weights = [m.get_num_samples() for m in models]
        params = weighted_mean([m.get_parameters() for m in models], weights)
        contributors: List[str] = []
        for m in models:
            contributors += m.get_contributors()
        return models[0].build_copy(params=params, num_samples=int(sum(weights)), contributors=contributors)
