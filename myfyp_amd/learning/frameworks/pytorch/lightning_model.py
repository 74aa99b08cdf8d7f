"""``LightningModel`` and the example ``MLP`` at their reference path
(``p2pfl/learning/frameworks/pytorch/lightning_model.py:37-207``).

``LightningModel`` is the reference name of the PyTorch model wrapper: parameters are the
``state_dict`` tensors in order (the pickle wire format), ``set_parameters`` checks shapes
(``ModelNotMatchingError``). Any ``torch.nn.Module`` works — it need not be a LightningModule;
the MLP here is a plain module returning log-probabilities, trained by the learner (Adam 1e-3,
the reference ``configure_optimizers``).
"""

from myfyp_amd.learning.frameworks.torch.torch_model import TorchModel
from myfyp_amd.models.mlp import MLP


class LightningModel(TorchModel):
    """Reference-named :class:`TorchModel` (same constructor: model, params, num_samples,
    contributors, additional_info, and the newer upstream's ``compression=`` dict — see
    :mod:`myfyp_amd.learning.compression`)."""

    def build_copy(self, **kwargs) -> "LightningModel":
        kwargs.setdefault("compression", self.compression)
        return LightningModel(None, _shapes=self.expected_shapes(), **kwargs)


__all__ = ["LightningModel", "MLP"]
