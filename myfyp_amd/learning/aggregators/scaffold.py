"""SCAFFOLD server side (parity: ``p2pfl/learning/aggregators/scaffold.py:29-139``).

``x ← x + η_g · Σ n_i Δy_i / Σ n_i`` and ``c ← c + mean(Δc_i)``; the result carries
``{"scaffold": {"global_c": c}}``. Difference: when no global model is tracked yet the reference
starts from the first *trained* model (``scaffold.py:88-90``); here it starts from that model's
round-start weights ``y_0 − Δy_0`` (the true global model).
"""

from __future__ import annotations

from typing import Any, List

import numpy as np

from myfyp_amd.learning.aggregators._math import to_numpy_list
from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class Scaffold(Aggregator):
    """Karimireddy et al., 2020 — https://arxiv.org/abs/1910.06378."""

    REQUIRED_INFO_KEYS = ["delta_y_i", "delta_c_i"]
    # collective plane: two device all-reduces (n-weighted Δy, mean Δc) + axpy, no host copies
    # (parallel/weights_plane.py: aggregate_scaffold)
    collective_kind = "scaffold"

    def __init__(self, node_name: str = "unknown", global_lr: float = 0.1) -> None:
        super().__init__(node_name)
        self.global_lr = global_lr
        self.c: List[np.ndarray] = []
        self.global_model_params: List[np.ndarray] = []
        self.partial_aggregation = False

    def aggregate(self, models: List[P2PFLModel]) -> P2PFLModel:
        if not models:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        total = sum(m.get_num_samples() for m in models)
        infos = [self._get_and_validate_model_info(m) for m in models]
        dys = [to_numpy_list(i["delta_y_i"]) for i in infos]
        dcs = [to_numpy_list(i["delta_c_i"]) for i in infos]
        acc_dy = [sum(dy[l] * m.get_num_samples() for dy, m in zip(dys, models)) / total * self.global_lr for l in range(len(dys[0]))]
        if not self.global_model_params:
            first = to_numpy_list(models[0].get_parameters())
            self.global_model_params = [p - d for p, d in zip(first, dys[0])]
        self.global_model_params = [np.asarray(p + d) for p, d in zip(self.global_model_params, acc_dy)]
        acc_c = [sum(dc[l] for dc in dcs) / len(dcs) for l in range(len(dcs[0]))]
        if not self.c:
            self.c = [np.zeros_like(a) for a in acc_c]
        self.c = [c + a for c, a in zip(self.c, acc_c)]
        contributors: List[str] = []
        for m in models:
            contributors.extend(m.get_contributors())
        out = models[0].build_copy(params=[p.copy() for p in self.global_model_params], num_samples=total, contributors=contributors)
        out.add_info("scaffold", {"global_c": [c.copy() for c in self.c]})
        return out

    def get_required_callbacks(self) -> List[str]:
        return ["scaffold"]

    def _get_and_validate_model_info(self, model: P2PFLModel) -> dict:
        info: Any = model.get_info().get("scaffold")
        if not isinstance(info, dict) or not all(k in info for k in self.REQUIRED_INFO_KEYS):
            raise ValueError(f"Model is missing required info keys: {self.REQUIRED_INFO_KEYS}")
        return info

    def clear(self) -> None:
        super().clear()
