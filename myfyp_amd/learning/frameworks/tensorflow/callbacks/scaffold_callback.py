"""Keras SCAFFOLD client (parity name: ``tensorflow/callbacks/scaffold_callback.py:30-163``).

The reference wraps the Keras optimizer to add ``c − c_i`` to every gradient. The MI355X stack
trains PyTorch models only; SCAFFOLD's client side is
:class:`~myfyp_amd.learning.frameworks.torch.callbacks.SCAFFOLDCallback` (correction fused into the
optimizer kernel). This name raises with that pointer.
"""

from __future__ import annotations


class ScaffoldOptimizerWrapper:
    def __init__(self, *args, **kwargs) -> None:
        raise NotImplementedError("ScaffoldOptimizerWrapper: Keras training is not part of the MI355X engine; use TorchLearner + SCAFFOLDCallback")


class SCAFFOLDCallback(ScaffoldOptimizerWrapper):
    """Reference callback name (Keras flavour)."""
