"""Decentralised neighbour averaging over a topology (BASELINE config 3: "gossip neighbor-avg
(ring topology) over xGMI"; D-PSGD, Lian et al. 2017 — https://arxiv.org/abs/1705.09056).

Every peer trains each round, then replaces its model with a doubly-stochastic mix of itself and
its topology neighbours: ``x_i ← Σ_j W_ij x_j`` with Metropolis–Hastings weights
``W_ij = 1 / (1 + max(deg_i, deg_j))`` (default) or uniform ``1 / (1 + deg_i)``. Unlike FedAvg the
peers do NOT agree after a round; they converge to consensus over rounds.

Collective plane (``collective_kind = "neighbor"``): co-located neighbours are mixed in place on
the GPU; neighbours on other ranks are exchanged with grouped RCCL ``send/recv`` over xGMI (one
model per cross-rank edge — for a ring split over N GPUs that is 2 models per GPU per round, no
all-reduce). Gossip plane (``aggregate``): the mean of the models it received (its neighbours').
"""

from __future__ import annotations

from typing import List

import numpy as np

from myfyp_amd.learning.aggregators._math import weighted_mean
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.utils.topologies import TopologyFactory, TopologyType


class NeighborAvg(Aggregator):
    collective_kind = "neighbor"
    all_peers_train = True  # no train-set vote: every peer trains every round

    def __init__(self, node_name: str = "unknown", topology: str = "ring", weights: str = "metropolis", adjacency=None) -> None:
        super().__init__(node_name)
        self.topology = topology
        self.weights = weights
        self.adjacency = None if adjacency is None else np.asarray(adjacency, dtype=int)
        self.partial_aggregation = True

    def adjacency_for(self, n: int) -> np.ndarray:
        if self.adjacency is not None:
            if self.adjacency.shape != (n, n):
                raise ValueError(f"adjacency is {self.adjacency.shape}, federation has {n} peers")
            return self.adjacency
        return TopologyFactory.generate_matrix(TopologyType(self.topology), n)

    def mixing_matrix(self, n: int) -> np.ndarray:
        a = self.adjacency_for(n).astype(bool)
        np.fill_diagonal(a, False)
        deg = a.sum(1)
        w = np.zeros((n, n), dtype=np.float64)
        for i in range(n):
            for j in np.nonzero(a[i])[0]:
                w[i, j] = 1.0 / (1 + max(deg[i], deg[j])) if self.weights == "metropolis" else 1.0 / (1 + deg[i])
            w[i, i] = 1.0 - w[i].sum()
        return w

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if not models:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        params = weighted_mean([m.get_parameters() for m in models], [1.0] * len(models))
        contributors: List[str] = []
        for m in models:
            contributors += m.get_contributors()
        return models[0].build_copy(params=params, num_samples=int(sum(m.get_num_samples() for m in models)), contributors=contributors)
