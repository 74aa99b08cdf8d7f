"""Parameter-format adapter for Keras models (see package docstring)."""

from __future__ import annotations

from typing import Any, List, Union

import numpy as np

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class ModelNotBuiltError(Exception):
    """A Keras model without weights (never built/called) was wrapped (reference ``keras_model.py:38``)."""


class KerasModel(P2PFLModel):
    """``get_weights()/set_weights()`` order, like the reference ``KerasModel``; works without
    TensorFlow when built from a parameter list (``KerasModel(None, params=[...])``)."""

    def __init__(self, model: Any = None, params=None, **kwargs) -> None:
        if model is not None and hasattr(model, "built") and not model.built:
            raise ModelNotBuiltError("The Keras model must be built (called once or given an input shape) before wrapping it")
        self._params: List[np.ndarray] = [np.asarray(w) for w in model.get_weights()] if model is not None else []
        super().__init__(model, params=params, **kwargs)

    def get_parameters(self) -> List[np.ndarray]:
        return [np.asarray(w) for w in self.model.get_weights()] if self.model is not None else self._params

    def set_parameters(self, params: Union[List[np.ndarray], bytes]) -> None:
        if isinstance(params, bytes):
            params, info = self.decode_parameters(params)
            self.additional_info.update(info)
        params = [np.asarray(p) for p in params]
        if self.model is not None:
            self.model.set_weights(params)
        self._params = params

    def build_copy(self, **kwargs) -> "P2PFLModel":
        return KerasModel(None, **kwargs)

    def get_framework(self) -> str:
        return Framework.TENSORFLOW.value
