"""Aggregator-required client callbacks for the PyTorch-ROCm learners.

Both work on the learner's flat parameter buffer and hand the optimizer kernel extra read streams
instead of editing gradients in Python:

* ``SCAFFOLDCallback`` (parity target: ``pytorch/callbacks/scaffold_callback.py:32-150``). The
  reference adds ``lr·(c_i − c)`` to ``param.grad`` of *detached state_dict copies*, so its
  correction is a no-op. Here the correction is real and applied in the UPDATE
  space of the local optimizer: ``w ← step(w, g) − lr·(c − c_i)`` (``opt_update``,
  ``csrc/kernels/common.h``; ``ops.adam_step``). The control variate follows SCAFFOLD option II,
  ``c_i⁺ = c_i − c + (x − y)/(K·lr)`` (the reference's formula, ``scaffold_callback.py:129``),
  which measures the mean local step in those same units — exact SCAFFOLD for plain SGD, and the
  consistent generalisation for Adam (the reference MLP's optimizer, ``lightning_model.py:181-183``)
  and momentum. Adding the correction to Adam's *gradient* instead (round 4) mixed normalised-step
  units into a gradient and the federation stopped learning (0.15–0.84 after two rounds); a
  gradient-unit control variate (option I, ∇f_i at the round-start model) fails the same test on
  all six seeds: with raw 0–255 inputs the first round's gradients dwarf the later ones, so the
  one-round-stale correction dominates the step.
* ``FedProxCallback``: proximal term ``μ(w − w_global)`` with ``w_global`` snapshotted at fit start.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np
import torch

from myfyp_amd.learning.frameworks.callback import P2PFLCallback
from myfyp_amd.learning.frameworks.callback_factory import CallbackFactory


class TorchCallback(P2PFLCallback):
    """Hook points used by the torch learners."""

    def on_train_start(self, learner) -> None: ...

    def grad_correction(self) -> Dict[str, Any]:
        return {}

    def on_train_end(self, learner, steps: int, lr: float) -> None: ...


def _flat_to_list(flat: torch.Tensor, learner) -> list:
    return [v.detach().cpu().numpy().copy() for v in learner.split_flat(flat)]


def _list_to_flat(arrs, like: torch.Tensor) -> torch.Tensor:
    if len(arrs) and isinstance(arrs[0], torch.Tensor):  # device-resident (collective plane)
        return torch.cat([a.detach().reshape(-1).to(device=like.device, dtype=torch.float32) for a in arrs])
    return torch.cat([torch.as_tensor(np.asarray(a), dtype=torch.float32).reshape(-1) for a in arrs]).to(like.device)


class SCAFFOLDCallback(TorchCallback):
    """Client side of SCAFFOLD."""

    def __init__(self) -> None:
        super().__init__()
        self.c_i: Optional[torch.Tensor] = None
        self.c: Optional[torch.Tensor] = None
        self.x0: Optional[torch.Tensor] = None
        self.delta_y: Optional[torch.Tensor] = None
        self.delta_c: Optional[torch.Tensor] = None

    @staticmethod
    def get_name() -> str:
        return "scaffold"

    def on_train_start(self, learner) -> None:
        flat = learner.flat_params()
        if self.c_i is None or self.c_i.numel() != flat.numel():
            self.c_i = torch.zeros_like(flat)
        elif self.c_i.device != flat.device:
            self.c_i = self.c_i.to(flat.device)
        g = self.additional_info.get("global_c")
        self.c = _list_to_flat(g, flat) if g is not None else torch.zeros_like(flat)
        self.x0 = flat.detach().clone()

    def grad_correction(self) -> Dict[str, Any]:
        return {"c_global": self.c, "c_local": self.c_i}

    def on_train_end(self, learner, steps: int, lr: float) -> None:
        assert self.x0 is not None and self.c_i is not None and self.c is not None
        y = learner.flat_params().detach()
        k = max(1, steps)
        c_new = self.c_i - self.c + (self.x0 - y) / (k * lr)
        # Δy / Δc stay device flats (one elementwise pass each, no host copy): the collective
        # SCAFFOLD reduction (weights_plane.aggregate_scaffold) all-reduces them on the GPU; the
        # per-layer entries are views of these flats, converted to numpy only at the wire boundary
        self.delta_y = y - self.x0
        self.delta_c = c_new - self.c_i
        self.c_i = c_new
        self.additional_info["delta_y_i"] = learner.split_flat(self.delta_y)
        self.additional_info["delta_c_i"] = learner.split_flat(self.delta_c)

    def state_dict(self) -> dict:
        return {} if self.c_i is None else {"c_i": self.c_i.detach().cpu().numpy()}

    def load_state_dict(self, state: dict) -> None:
        if "c_i" in state:
            self.c_i = torch.as_tensor(np.asarray(state["c_i"]), dtype=torch.float32)


class FedProxCallback(TorchCallback):
    """Client side of FedProx."""

    def __init__(self) -> None:
        super().__init__()
        self.anchor: Optional[torch.Tensor] = None

    @staticmethod
    def get_name() -> str:
        return "fedprox"

    def on_train_start(self, learner) -> None:
        self.anchor = learner.flat_params().detach().clone()

    def grad_correction(self) -> Dict[str, Any]:
        return {"anchor": self.anchor, "mu": float(self.additional_info.get("mu", 0.01))}


for _fw in ("pytorch", "rocm"):
    CallbackFactory.register_callback(_fw, SCAFFOLDCallback)
    CallbackFactory.register_callback(_fw, FedProxCallback)
