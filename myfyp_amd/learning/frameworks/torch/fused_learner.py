"""``Framework.ROCM`` learner: a ``TorchLearner`` that REQUIRES the fused grouped engine."""

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner


class FusedMLPLearner(TorchLearner):
    """Fails loudly if the model/device cannot run on the fused HIP engine."""

    def _maybe_attach_engine(self, module):
        eng = super()._maybe_attach_engine(module)
        if eng is None:
            raise RuntimeError("FusedMLPLearner needs a ReLU MLP on an MI355X with the native library built")
        return eng

    def get_framework(self) -> str:
        return Framework.ROCM.value
