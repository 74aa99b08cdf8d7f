"""``FlaxExportStrategy`` (parity: ``flax/flax_dataset.py:30-67``): ``(x, y)`` NumPy batches
(JAX consumes NumPy arrays directly; JAX itself is not part of the MI355X stack)."""

from __future__ import annotations

from typing import Any, Callable, Optional

from myfyp_amd.learning.dataset.p2pfl_dataset import DataExportStrategy
from myfyp_amd.learning.frameworks._numpy_export import NumpyBatches


class FlaxExportStrategy(DataExportStrategy):
    @staticmethod
    def export(data: Any, transforms: Optional[Callable] = None, train: bool = True, batch_size: int = 1, **kwargs) -> Any:
        return NumpyBatches(data, train, batch_size, shuffle=train, transforms=transforms)
