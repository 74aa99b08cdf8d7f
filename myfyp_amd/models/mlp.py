"""Multilayer perceptron (parity: ``p2pfl/learning/frameworks/pytorch/lightning_model.py:118-207``).

Same layer list (``layers = [Linear, act, Linear, act, ..., Linear]``), so the ``state_dict`` order —
and therefore the wire format — matches the reference: ``layers.0.weight, layers.0.bias,
layers.2.weight, ...``. Inputs are raw ``uint8`` images cast to float (no normalisation), output is
``log_softmax``. With ReLU activations on a GPU the whole train step (fwd + bwd + Adam) runs in the
fused HIP engine (:mod:`myfyp_amd.parallel.mlp_engine`).
"""

from __future__ import annotations

from typing import List, Optional

import torch


class MLP(torch.nn.Module):
    """``input_size → hidden_sizes... → out_channels`` with a configurable activation."""

    def __init__(
        self,
        input_size: int = 28 * 28,
        hidden_sizes: Optional[List[int]] = None,
        out_channels: int = 10,
        activation: str = "relu",
        lr_rate: float = 0.001,
        seed: Optional[int] = None,
    ) -> None:
        super().__init__()
        hidden_sizes = [256, 128] if hidden_sizes is None else list(hidden_sizes)
        if seed is not None:
            torch.manual_seed(seed)
        self.input_size = input_size
        self.hidden_sizes = hidden_sizes
        self.out_channels = out_channels
        self.activation = activation
        self.lr_rate = lr_rate
        dims = [input_size] + hidden_sizes
        self.layers = torch.nn.ModuleList()
        for i in range(len(hidden_sizes)):
            self.layers.append(torch.nn.Linear(dims[i], dims[i + 1]))
            self.layers.append(self._get_activation(activation))
        self.layers.append(torch.nn.Linear(hidden_sizes[-1], out_channels))

    @staticmethod
    def _get_activation(name: str) -> torch.nn.Module:
        if name == "relu":
            return torch.nn.ReLU()
        if name == "sigmoid":
            return torch.nn.Sigmoid()
        if name == "tanh":
            return torch.nn.Tanh()
        raise ValueError(f"Unsupported activation function: {name}")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.reshape(x.shape[0], -1).float()
        for layer in self.layers:
            x = layer(x)
        return torch.log_softmax(x, dim=1)

    def optimizer_spec(self) -> dict:
        """Optimizer used by the learner (reference: ``torch.optim.Adam(lr=lr_rate)``)."""
        return {"name": "adam", "lr": self.lr_rate}

    def linear_layers(self) -> List[torch.nn.Linear]:
        return [m for m in self.layers if isinstance(m, torch.nn.Linear)]
