"""Dataset export for PyTorch (parity: ``frameworks/pytorch/lightning_dataset.py``:
``PyTorchExportStrategy`` and ``TorchvisionDatasetFactory``).

``PyTorchExportStrategy.export(data, batch_size=1)`` returns a ``torch.utils.data.DataLoader`` over a
:class:`~myfyp_amd.learning.dataset.p2pfl_dataset.P2PFLDataset` split (reference default batch 1).
The learners themselves do not use it — they keep each peer's split resident on the GPU — but it is
the public way to hand a partition to ordinary PyTorch code.
``TorchvisionDatasetFactory.get_mnist`` builds a P2PFLDataset from a torchvision MNIST directory
already on disk (nothing is downloaded).
"""

from __future__ import annotations

import os
from typing import Any, Callable, Optional

import numpy as np
import torch

from myfyp_amd.learning.dataset.p2pfl_dataset import DataExportStrategy, P2PFLDataset


class _SplitDataset(torch.utils.data.Dataset):
    def __init__(self, data: P2PFLDataset, train: bool, transforms: Optional[Callable]) -> None:
        self.x = data.column("image", train)
        self.y = data.column("label", train)
        self.transforms = transforms

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, i: int):
        item = {"image": torch.from_numpy(np.asarray(self.x[i])), "label": int(self.y[i])}
        return self.transforms(item) if self.transforms is not None else item


class PyTorchExportStrategy(DataExportStrategy):
    @staticmethod
    def export(data: Any, transforms: Optional[Callable] = None, train: bool = True, batch_size: int = 1, num_workers: int = 0, **kwargs) -> Any:
        if not isinstance(data, P2PFLDataset):
            raise TypeError("PyTorchExportStrategy exports P2PFLDataset splits")
        ds = _SplitDataset(data, train, transforms or data.get_transforms())
        return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=train, num_workers=num_workers)


class TorchvisionDatasetFactory:
    """Local torchvision datasets → P2PFLDataset (no download: the build/GPU hosts have no network)."""

    @staticmethod
    def get_mnist(cache_dir: str = "./data", train: bool = True, download: bool = False) -> P2PFLDataset:
        import torchvision  # optional

        if download:
            raise RuntimeError("downloads are not available; place the MNIST files under cache_dir")
        if not os.path.isdir(cache_dir):
            raise FileNotFoundError(cache_dir)
        tr = torchvision.datasets.MNIST(cache_dir, train=True, download=False)
        te = torchvision.datasets.MNIST(cache_dir, train=False, download=False)
        return P2PFLDataset.from_arrays(
            {"image": tr.data.numpy().astype(np.uint8), "label": tr.targets.numpy().astype(np.int64)},
            {"image": te.data.numpy().astype(np.uint8), "label": te.targets.numpy().astype(np.int64)},
        )
