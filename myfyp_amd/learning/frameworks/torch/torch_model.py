"""PyTorch-ROCm model wrapper (parity: ``p2pfl/learning/frameworks/pytorch/lightning_model.py:37-108``).

``get_parameters`` returns the ``state_dict`` as numpy arrays in order (wire format);
``set_parameters`` checks count/shapes (``ModelNotMatchingError``) and copies in place so a
device-resident module (and its flat buffer) is never reallocated.

``build_copy`` is *parameter-only* (no ``deepcopy`` of the module, which the reference does per
received partial model, ``partial_model_command.py:80``): copies are containers for aggregation;
learners copy their values into their own live module (``TorchLearner.set_model``).
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

import numpy as np
import torch

from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.exceptions import ModelNotMatchingError
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class TorchModel(P2PFLModel):
    """Wraps a ``torch.nn.Module`` (or, for copies, just its parameter list)."""

    def __init__(
        self,
        model: Optional[torch.nn.Module],
        params: Optional[Union[List[np.ndarray], bytes]] = None,
        num_samples: Optional[int] = None,
        contributors: Optional[List[str]] = None,
        additional_info: Optional[Dict[str, Any]] = None,
        _shapes: Optional[List[tuple]] = None,
        compression: Optional[Dict[str, Any]] = None,
    ) -> None:
        self._params: Optional[List[np.ndarray]] = None
        self._shapes = _shapes
        super().__init__(model, params, num_samples, contributors, additional_info, compression=compression)

    # ------------------------------------------------------------------ params
    def _state_tensors(self) -> List[torch.Tensor]:
        assert self.model is not None
        return list(self.model.state_dict().values())

    def get_parameters(self) -> List[np.ndarray]:
        if self.model is None:
            return self._params or []
        return [t.detach().cpu().numpy() for t in self._state_tensors()]

    def get_tensors(self) -> List[torch.Tensor]:
        """Live state tensors (device-resident, no copy)."""
        if self.model is None:
            return [torch.from_numpy(np.ascontiguousarray(p)) for p in (self._params or [])]
        return [t.detach() for t in self._state_tensors()]

    def expected_shapes(self) -> Optional[List[tuple]]:
        if self.model is not None:
            return [tuple(t.shape) for t in self._state_tensors()]
        return self._shapes

    def set_parameters(self, params: Union[List[np.ndarray], List[torch.Tensor], bytes]) -> None:
        if isinstance(params, (bytes, bytearray)):
            params, info = self.decode_parameters(bytes(params))
            self.additional_info.update(info)
        params = list(params)
        shapes = self.expected_shapes()
        if shapes is not None:
            if len(params) != len(shapes):
                raise ModelNotMatchingError(f"Expected {len(shapes)} tensors, got {len(params)}")
            for p, s in zip(params, shapes):
                if tuple(np.shape(p)) != tuple(s):
                    raise ModelNotMatchingError(f"Shape mismatch: {tuple(np.shape(p))} vs {tuple(s)}")
        if self.model is None:
            self._params = [p.detach().cpu().numpy() if isinstance(p, torch.Tensor) else np.asarray(p) for p in params]
            if self._shapes is None:
                self._shapes = [tuple(p.shape) for p in self._params]
            return
        with torch.no_grad():
            for dst, src in zip(self._state_tensors(), params):
                src_t = src if isinstance(src, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(src))
                dst.copy_(src_t.to(dst.dtype), non_blocking=False)

    def build_copy(self, **kwargs) -> "TorchModel":
        kwargs.setdefault("compression", self.compression)
        return TorchModel(None, _shapes=self.expected_shapes(), **kwargs)

    def get_framework(self) -> str:
        return Framework.PYTORCH.value
