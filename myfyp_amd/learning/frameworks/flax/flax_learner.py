"""``FlaxLearner`` (parity name: ``flax/flax_learner.py:40-181``). JAX/Flax training is outside the
MI355X stack; the class raises with a pointer to the interop path (``FlaxModel`` parameter leaves in
the wire format → a TorchModel of the same architecture)."""

from __future__ import annotations

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.learner import Learner

_MSG = "FlaxLearner: JAX training is not part of the MI355X engine; load FlaxModel's parameters into a TorchModel and train with TorchLearner."


class FlaxLearner(Learner):
    def __init__(self, *args, **kwargs) -> None:
        raise NotImplementedError(_MSG)

    def fit(self):  # pragma: no cover
        raise NotImplementedError(_MSG)

    def interrupt_fit(self) -> None:  # pragma: no cover
        raise NotImplementedError(_MSG)

    def evaluate(self):  # pragma: no cover
        raise NotImplementedError(_MSG)

    def get_framework(self) -> str:
        return Framework.FLAX.value
