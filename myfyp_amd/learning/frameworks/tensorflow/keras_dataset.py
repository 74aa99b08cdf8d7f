"""``KerasExportStrategy`` (parity: ``tensorflow/keras_dataset.py:29-69``).

The reference returns a ``tf.data.Dataset`` of ``(image, label)`` batches (batch 1 by default). With
no TensorFlow in the MI355X stack the same batches come back as NumPy arrays, which
``keras.Model.fit`` accepts directly and which any host-side tool can consume.
"""

from __future__ import annotations

from typing import Any, Callable, Optional

from myfyp_amd.learning.dataset.p2pfl_dataset import DataExportStrategy
from myfyp_amd.learning.frameworks._numpy_export import NumpyBatches


class KerasExportStrategy(DataExportStrategy):
    @staticmethod
    def export(data: Any, transforms: Optional[Callable] = None, train: bool = True, batch_size: int = 1, **kwargs) -> Any:
        return NumpyBatches(data, train, batch_size, shuffle=train, transforms=transforms)
