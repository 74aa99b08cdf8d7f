"""``LightningLearner`` at its reference path (``pytorch/lightning_learner.py:43-152``).

Same constructor ``(model, data, self_addr, aggregator)`` and methods (``fit``, ``interrupt_fit``,
``evaluate``, ``get_framework``); training runs on :class:`TorchLearner`'s GPU path instead of a
Lightning ``Trainer`` (one fused Adam launch per step, or the grouped fused-MLP engine).
"""

from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner


class LightningLearner(TorchLearner):
    """Reference-named :class:`TorchLearner`."""


__all__ = ["LightningLearner"]
