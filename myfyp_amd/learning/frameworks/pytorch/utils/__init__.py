"""PyTorch dataset utilities (reference: ``pytorch/utils/``)."""
