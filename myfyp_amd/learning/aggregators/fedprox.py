"""FedProx (Li et al., 2020). Server side = FedAvg; client side adds ``μ(w − w_global)`` to the
gradient, which the learner fuses into the optimizer kernel. The aggregator
requires the ``fedprox`` callback and ships ``μ`` through ``additional_info``."""

from __future__ import annotations

from typing import List

from myfyp_amd.learning.aggregators.fedavg import FedAvg
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class FedProx(FedAvg):
    """FedAvg + proximal-term client callback."""

    def __init__(self, node_name: str = "unknown", proximal_mu: float = 0.01) -> None:
        super().__init__(node_name)
        self.proximal_mu = proximal_mu

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        out = super().aggregate(models)
        out.add_info("fedprox", {"mu": self.proximal_mu})
        return out

    def get_required_callbacks(self) -> List[str]:
        return ["fedprox"]
