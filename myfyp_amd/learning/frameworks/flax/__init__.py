"""Flax interop (parity names only: ``frameworks/flax/flax_model.py``): ``FlaxModel`` carries a
parameter pytree's leaves in the shared wire format; there is no JAX training path on MI355X."""

from myfyp_amd.learning.frameworks.flax.flax_model import FlaxModel

__all__ = ["FlaxModel"]
