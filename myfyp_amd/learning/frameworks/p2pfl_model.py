"""Framework-neutral model wrapper and the wire/checkpoint format.

Parity: ``p2pfl/learning/frameworks/p2pfl_model.py:30-195``. The serialized format is unchanged:
``pickle.dumps({"params": List[np.ndarray] (state_dict order), "additional_info": {...}})`` so peers
and checkpoints interoperate with the reference. Decoding uses a restricted unpickler that only
materialises numpy arrays and plain containers (no arbitrary code execution from the network).
"""

from __future__ import annotations

import copy
import io
import pickle
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np

from myfyp_amd.learning.frameworks.exceptions import DecodingParamsError
from myfyp_amd.management.tracing import traced

_SAFE_GLOBALS = {
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"),
    ("numpy.core.numeric", "_frombuffer"),
    ("numpy._core.numeric", "_frombuffer"),
    ("builtins", "complex"),
    ("builtins", "bytearray"),
    ("collections", "OrderedDict"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str) -> Any:
        if (module, name) in _SAFE_GLOBALS or (module.startswith("numpy") and name.endswith("DType")):
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"Refusing to unpickle {module}.{name}")


def safe_loads(data: bytes) -> Any:
    """Unpickle model payloads allowing only numpy arrays and builtin containers."""
    return _SafeUnpickler(io.BytesIO(data)).load()


def _to_host(obj: Any) -> Any:
    """Callback info may hold device tensors (SCAFFOLD Δy/Δc stay on the GPU between rounds); the
    wire/checkpoint format carries numpy arrays only — converted here, at the boundary."""
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    if type(obj).__module__.startswith("torch") and hasattr(obj, "detach"):
        return obj.detach().cpu().numpy()
    return obj


class P2PFLModel:
    """Holds parameters (as numpy on the wire), contributors, sample count and callback info."""

    def __init__(
        self,
        model: Any,
        params: Optional[Union[List[np.ndarray], bytes]] = None,
        num_samples: Optional[int] = None,
        contributors: Optional[List[str]] = None,
        additional_info: Optional[Dict[str, Any]] = None,
        compression: Optional[Dict[str, Any]] = None,
    ) -> None:
        from myfyp_amd.learning import compression as _comp

        self.model = model
        # wire compression of this model's payloads (learning/compression.py; None = reference format)
        self.compression = _comp.validate(compression)
        self.contributors: List[str] = list(contributors) if contributors is not None else []
        self.num_samples: int = num_samples if num_samples is not None else 0
        self.additional_info: Dict[str, Any] = additional_info if additional_info is not None else {}
        if params is not None:
            self.set_parameters(params)

    def get_model(self) -> Any:
        return self.model

    # ------------------------------------------------------------------ wire format
    @traced("encode")
    def encode_parameters(self, params: Optional[List[np.ndarray]] = None) -> bytes:
        from myfyp_amd.learning import compression as _comp

        if params is None:
            params = self.get_parameters()
        return _comp.encode(params, _to_host(self.additional_info), getattr(self, "compression", None))

    def decode_parameters(self, data: bytes) -> Tuple[List[np.ndarray], Dict[str, Any]]:
        """Reference payloads and compressed ones (``learning/compression.py``) alike."""
        from myfyp_amd.learning import compression as _comp

        try:
            shapes_of = getattr(self, "expected_shapes", None)
            shapes = shapes_of() if callable(shapes_of) else None
            return _comp.decode(data, safe_loads, shapes)
        except Exception as e:
            raise DecodingParamsError("Error decoding parameters") from e

    # ------------------------------------------------------------------ parameters
    def get_parameters(self) -> List[np.ndarray]:
        raise NotImplementedError

    def set_parameters(self, params: Union[List[np.ndarray], bytes]) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------ info / contribution
    def add_info(self, callback: str, info: Any) -> None:
        self.additional_info[callback] = info

    def get_info(self, callback: Optional[str] = None) -> Any:
        if callback is None:
            return self.additional_info
        return self.additional_info[callback]

    def set_contribution(self, contributors: List[str], num_samples: int) -> None:
        self.contributors = list(contributors)
        self.num_samples = num_samples

    def get_contributors(self) -> List[str]:
        if not self.contributors:
            raise ValueError("Contributors are empty")
        return self.contributors

    def get_num_samples(self) -> int:
        if self.num_samples == 0:
            raise ValueError("Number of samples required")
        return self.num_samples

    def build_copy(self, **kwargs) -> "P2PFLModel":
        return self.__class__(copy.deepcopy(self.model), **kwargs)

    def get_framework(self) -> str:
        raise NotImplementedError


class NumpyModel(P2PFLModel):
    """Parameter-only model (aggregation math, interop with non-PyTorch peers, tests)."""

    def __init__(self, model: Any = None, params=None, **kwargs) -> None:
        self._params: List[np.ndarray] = []
        super().__init__(model, params=params, **kwargs)

    def get_parameters(self) -> List[np.ndarray]:
        return self._params

    def set_parameters(self, params: Union[List[np.ndarray], bytes]) -> None:
        if isinstance(params, bytes):
            params, info = self.decode_parameters(params)
            self.additional_info.update(info)
        self._params = [np.asarray(p) for p in params]

    def build_copy(self, **kwargs) -> "P2PFLModel":
        return NumpyModel(None, **kwargs)

    def get_framework(self) -> str:
        return "numpy"
