"""Keras callbacks (reference: ``tensorflow/callbacks/``)."""
