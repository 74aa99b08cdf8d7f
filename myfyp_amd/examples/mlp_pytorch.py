"""The FYP's MLP model module (``/root/reference/mlp_pytorch.txt``) as a ``model_build_fn`` package.

YAML configs name it the way the FYP does::

    model:
      package: myfyp_amd.examples.mlp_pytorch
      model_build_fn: model_build_fn
      params: {hidden_sizes: [256, 128], compression: {ptq: {dtype: float16}, zlib: {level: 6}}}

``compression`` (``mlp_pytorch.txt:148-151`` pops it before building the MLP) selects the wire
compression of the model's payloads — see :mod:`myfyp_amd.learning.compression`.
"""

from __future__ import annotations

from myfyp_amd.learning.frameworks.pytorch.lightning_model import LightningModel
from myfyp_amd.models import MLP


def model_build_fn(*args, **kwargs) -> LightningModel:
    compression = kwargs.pop("compression", None)
    return LightningModel(MLP(*args, **kwargs), compression=compression)


__all__ = ["MLP", "model_build_fn"]
