"""PyTorch callbacks at their reference path (``pytorch/callbacks/``)."""
