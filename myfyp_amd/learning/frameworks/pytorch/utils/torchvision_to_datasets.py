"""torchvision dataset → Hugging Face ``datasets`` (parity: ``pytorch/utils/torchvision_to_datasets.py``).

The reference builds a ``DatasetDict`` from a torchvision dataset and pushes it to the HF Hub. With
no network here the result is returned (and optionally saved with ``save_to_disk``) so it can be
loaded with :meth:`P2PFLDataset.from_huggingface` / ``datasets.load_from_disk`` on any host.

    python -m myfyp_amd.learning.frameworks.pytorch.utils.torchvision_to_datasets --root ./data --dataset MNIST --out ./mnist_hf
"""

from __future__ import annotations

import argparse
from typing import Any, Dict, Optional

import numpy as np


def _split_arrays(ds: Any) -> Dict[str, np.ndarray]:
    data = getattr(ds, "data", None)
    targets = getattr(ds, "targets", None)
    if data is not None and targets is not None:
        x = data.numpy() if hasattr(data, "numpy") else np.asarray(data)
        y = targets.numpy() if hasattr(targets, "numpy") else np.asarray(targets)
    else:  # generic (image, label) dataset
        pairs = [ds[i] for i in range(len(ds))]
        x = np.stack([np.asarray(p[0]) for p in pairs])
        y = np.asarray([int(p[1]) for p in pairs])
    return {"image": x.astype(np.uint8), "label": y.astype(np.int64)}


def create_huggingface_dataset_from_torchvision(train_dataset: Any, test_dataset: Any, save_path: Optional[str] = None):
    """Two torchvision datasets → ``datasets.DatasetDict({"train", "test"})`` with ``image``/``label``
    columns (images kept as uint8 arrays, the layout the learners upload to HBM)."""
    import datasets

    out = {}
    for split, ds in (("train", train_dataset), ("test", test_dataset)):
        cols = _split_arrays(ds)
        out[split] = datasets.Dataset.from_dict({"image": list(cols["image"]), "label": cols["label"].tolist()})
    dd = datasets.DatasetDict(out)
    if save_path:
        dd.save_to_disk(save_path)
    return dd


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--root", required=True, help="directory holding the torchvision files (no download)")
    ap.add_argument("--dataset", default="MNIST", help="torchvision.datasets class name")
    ap.add_argument("--out", required=True, help="save_to_disk destination")
    a = ap.parse_args(argv)
    import torchvision

    cls = getattr(torchvision.datasets, a.dataset)
    create_huggingface_dataset_from_torchvision(cls(a.root, train=True, download=False), cls(a.root, train=False, download=False), a.out)


if __name__ == "__main__":
    main()
