"""(Multi-)Krum (Blanchard et al., 2017): robust selection for the FYP Byzantine harness
(``exp_SAVE3.txt:60-234``). Not in the reference."""

from __future__ import annotations

from typing import List

import numpy as np

from myfyp_amd.learning.aggregators._math import _is_torch, flatten, weighted_mean
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class Krum(Aggregator):
    """Score each model by the summed squared distance to its ``n - f - 2`` nearest peers; average
    the ``m`` best (m=1 → classic Krum)."""

    collective_kind = None

    def __init__(self, node_name: str = "unknown", num_byzantine: int = 1, multi: int = 1) -> None:
        super().__init__(node_name)
        self.f = num_byzantine
        self.m = multi
        self.partial_aggregation = False

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if not models:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        n = len(models)
        flats = [flatten(m.get_parameters()) for m in models]
        if _is_torch(flats[0]):
            import torch

            X = torch.stack(flats)
            d = torch.cdist(X, X).pow(2).cpu().numpy()
        else:
            X = np.stack(flats)
            sq = (X * X).sum(1)
            d = np.maximum(sq[:, None] + sq[None, :] - 2 * X @ X.T, 0)
        k = max(1, n - self.f - 2)
        scores = [np.sort(np.delete(d[i], i))[:k].sum() for i in range(n)]
        chosen = [models[i] for i in np.argsort(scores)[: max(1, min(self.m, n))]]
        params = weighted_mean([m.get_parameters() for m in chosen], [m.get_num_samples() for m in chosen])
        contributors: List[str] = []
        for m in models:
            contributors += m.get_contributors()
        return models[0].build_copy(params=params, num_samples=sum(m.get_num_samples() for m in models), contributors=contributors)
