"""``KerasLearner`` (parity name: ``tensorflow/keras_learner.py:36-124``).

Training Keras models is outside the MI355X stack (PyTorch-ROCm only, no multi-backend
dispatch). The class exists so reference code that names it fails with an actionable message
instead of an ``ImportError``; Keras peers' *parameters* still interoperate through
:class:`~myfyp_amd.learning.frameworks.tensorflow.keras_model.KerasModel` (wire format).
"""

from __future__ import annotations

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.learner import Learner

_MSG = (
    "KerasLearner: TensorFlow training is not part of the MI355X engine. Load the Keras model's "
    "parameters into a TorchModel of the same architecture (KerasModel carries them in the wire format) "
    "and train it with TorchLearner."
)


class KerasLearner(Learner):
    def __init__(self, *args, **kwargs) -> None:
        raise NotImplementedError(_MSG)

    def fit(self):  # pragma: no cover - unreachable
        raise NotImplementedError(_MSG)

    def interrupt_fit(self) -> None:  # pragma: no cover
        raise NotImplementedError(_MSG)

    def evaluate(self):  # pragma: no cover
        raise NotImplementedError(_MSG)

    def get_framework(self) -> str:
        return Framework.TENSORFLOW.value
