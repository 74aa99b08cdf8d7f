"""Keras interop (parity names only: ``frameworks/tensorflow/keras_model.py``).

There is no TensorFlow training path on MI355X (PyTorch-ROCm only — no multi-backend dispatch).
``KerasModel`` carries a Keras model's weights in the shared wire format so Keras peers' models can
be aggregated, checkpointed and converted; ``LearnerFactory`` refuses to *train* it.
"""

from myfyp_amd.learning.frameworks.tensorflow.keras_model import KerasModel

__all__ = ["KerasModel"]
