"""Dataset export at its reference path (``pytorch/lightning_dataset.py:31-103``):
``PyTorchExportStrategy`` (DataLoader over a partition, batch 1 by default) and
``TorchvisionDatasetFactory`` (local torchvision files → P2PFLDataset, no download)."""

from myfyp_amd.learning.frameworks.torch.export import PyTorchExportStrategy, TorchvisionDatasetFactory

__all__ = ["PyTorchExportStrategy", "TorchvisionDatasetFactory"]
