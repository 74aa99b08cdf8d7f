"""Model zoo: the reference MLP (``lightning_model.py:118-207``), LeNet-5 and ResNet-18 (BASELINE
configs 3-5). All are plain ``torch.nn.Module``s whose ``forward`` returns log-probabilities, like
the reference MLP, so ``F.cross_entropy(model(x), y)`` is exactly the reference loss."""

from myfyp_amd.models.cnn import LeNet5, ResNet18
from myfyp_amd.models.mlp import MLP

__all__ = ["MLP", "LeNet5", "ResNet18"]
