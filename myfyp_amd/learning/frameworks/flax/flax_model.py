"""Parameter-format adapter for Flax parameter pytrees (leaves in tree-flatten order)."""

from __future__ import annotations

from typing import Any, List, Union

import numpy as np

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


def _leaves(tree: Any) -> List[Any]:
    if isinstance(tree, dict):
        return [leaf for k in sorted(tree) for leaf in _leaves(tree[k])]
    if isinstance(tree, (list, tuple)):
        return [leaf for t in tree for leaf in _leaves(t)]
    return [tree]


def _rebuild(tree: Any, leaves: List[np.ndarray]) -> Any:
    if isinstance(tree, dict):
        return {k: _rebuild(tree[k], leaves) for k in sorted(tree)}
    if isinstance(tree, (list, tuple)):
        return type(tree)(_rebuild(t, leaves) for t in tree)
    return leaves.pop(0)


class FlaxModel(P2PFLModel):
    """``model`` is ignored for training; ``init_params`` is the (nested dict) parameter pytree."""

    def __init__(self, model: Any = None, init_params: Any = None, params=None, **kwargs) -> None:
        self.tree = init_params
        super().__init__(model, params=params, **kwargs)

    def get_parameters(self) -> List[np.ndarray]:
        return [np.asarray(x) for x in _leaves(self.tree)] if self.tree is not None else []

    def set_parameters(self, params: Union[List[np.ndarray], bytes]) -> None:
        if isinstance(params, bytes):
            params, info = self.decode_parameters(params)
            self.additional_info.update(info)
        leaves = [np.asarray(p) for p in params]
        self.tree = _rebuild(self.tree, list(leaves)) if self.tree is not None else leaves

    def build_copy(self, **kwargs) -> "P2PFLModel":
        return FlaxModel(None, init_params=self.tree, **kwargs)

    def get_framework(self) -> str:
        return Framework.FLAX.value
