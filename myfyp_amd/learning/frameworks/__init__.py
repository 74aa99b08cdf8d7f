"""Framework identifiers (parity: ``p2pfl/learning/frameworks/__init__.py:14-19``).

``PYTORCH`` is the PyTorch-ROCm learner (autograd + fused HIP optimizer/aggregation kernels);
``ROCM`` is the fully fused native engine (hand-written HIP fwd/bwd/optimizer, hipGraph-replayed
epochs, grouped co-located peers). TensorFlow/Flax identifiers are kept so configs that name them
fail with a clear message instead of an import error (no multi-backend dispatch on MI355X).
"""

from enum import Enum


class Framework(Enum):
    PYTORCH = "pytorch"
    ROCM = "rocm"
    TENSORFLOW = "tensorflow"
    FLAX = "flax"
