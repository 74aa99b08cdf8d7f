"""PyTorch-ROCm framework integration: ``TorchModel``, ``TorchLearner``, callbacks."""

from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
from myfyp_amd.learning.frameworks.torch.torch_model import TorchModel

__all__ = ["TorchModel", "TorchLearner"]
