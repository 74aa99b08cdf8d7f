"""``model.get_framework() → Learner class`` (parity: ``frameworks/learner_factory.py:29-56``)."""

from __future__ import annotations

from typing import Type

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.learner import Learner
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class LearnerFactory:
    """Chooses the learner for a model."""

    @staticmethod
    def create_learner(model: P2PFLModel) -> Type[Learner]:
        fw = model.get_framework()
        if fw == Framework.PYTORCH.value:
            from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner

            return TorchLearner
        if fw == Framework.ROCM.value:
            from myfyp_amd.learning.frameworks.torch.fused_learner import FusedMLPLearner

            return FusedMLPLearner
        if fw in (Framework.TENSORFLOW.value, Framework.FLAX.value):
            raise ValueError(
                f"Framework {fw!r} is not supported by the MI355X engine (PyTorch-ROCm only). "
                "Export the model's parameters (P2PFLModel wire format) and load them into a TorchModel."
            )
        raise ValueError(f"Unsupported framework: {fw}")
