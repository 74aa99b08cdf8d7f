"""torchvision dataset → Hugging Face ``datasets`` (parity: ``pytorch/utils/torchvision_to_datasets.py``).

The reference builds a ``DatasetDict`` from a torchvision dataset, pushes it to the HF Hub and
pushes a dataset card rendered from a template (``torchvision_to_datasets.py:141-183``). Here:

* :func:`create_huggingface_dataset_from_torchvision` builds the ``DatasetDict`` (and optionally
  ``save_to_disk``s it, for hosts without a network: load it with ``datasets.load_from_disk`` or
  :meth:`P2PFLDataset.from_huggingface`);
* :func:`push_to_hub` logs in, pushes the splits, renders ``dataset_card_template.md`` with the
  card fields (language, license, task, pretty name, summary, description, source link) and pushes
  the card. The existing card's metadata is merged in when the Hub has one (the reference requires
  it). No network in this environment: the push path is exercised against a stand-in Hub client in
  ``tests/test_runtime_features.py`` (parity unpinned).

    python -m myfyp_amd.learning.frameworks.pytorch.utils.torchvision_to_datasets --root ./data --dataset MNIST --out ./mnist_hf
    ... --push --repo-id MNIST --token hf_... --license mit --official-link http://yann.lecun.com/exdb/mnist/
"""

from __future__ import annotations

import argparse
import os
import shutil
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


SUPPORTED_DATASETS = ("CIFAR10", "CIFAR100", "MNIST", "FashionMNIST", "EMNIST", "QMNIST")
TEMPLATE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dataset_card_template.md")


def dataset_card(name: str, license: Optional[str] = None, official_link: Optional[str] = None, summary: Optional[str] = None,
                 description: Optional[str] = None, base: Optional[Dict[str, Any]] = None, template_path: str = TEMPLATE):
    """The dataset card the push publishes: ``base`` (existing card metadata, if any) updated with
    the image-classification fields, rendered from ``template_path``."""
    from huggingface_hub import DatasetCard, DatasetCardData

    data = dict(base or {})
    data.update({"language": "en", "task_categories": ["image-classification"], "task_ids": ["multi-class-image-classification"],
                 "multilinguality": "monolingual", "pretty_name": name})
    if license:
        data["license"] = license
    source = f"Built from torchvision's {name}; see the original [{name}]({official_link})." if official_link else None
    return DatasetCard.from_template(card_data=DatasetCardData(**data), template_path=template_path, dataset_summary=summary,
                                     dataset_description=description, source_data=source, license=license)


def push_to_hub(dd, repo_id: str, token: Optional[str] = None, public: bool = False, license: Optional[str] = None,
                official_link: Optional[str] = None, summary: Optional[str] = None, description: Optional[str] = None, api=None) -> str:
    """Push ``dd`` (a ``DatasetDict``) and its card to ``repo_id``; returns the full repo name.
    ``api`` is the ``huggingface_hub`` module (or a stand-in with ``login``, ``get_full_repo_name``)."""
    if api is None:
        import huggingface_hub as api
    if token:
        api.login(token)
    dd.push_to_hub(repo_id=repo_id, private=not public, token=token)
    full = api.get_full_repo_name(repo_id, token=token) if "/" not in repo_id else repo_id
    base: Dict[str, Any] = {}
    try:  # the card the dataset push created (metadata: splits, features, sizes)
        from huggingface_hub import DatasetCard

        base = DatasetCard.load(full, token=token).data.to_dict()
    except Exception:
        base = {}
    card = dataset_card(repo_id.split("/")[-1], license, official_link, summary, description, base)
    card.push_to_hub(full, repo_type="dataset", token=token)
    return full


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--root", required=True, help="directory holding the torchvision files (no download)")
    ap.add_argument("--dataset", default="MNIST", help="torchvision.datasets class name")
    ap.add_argument("--out", default=None, help="save_to_disk destination")
    ap.add_argument("--push", action="store_true", help="push the splits and a dataset card to the HF Hub")
    ap.add_argument("--repo-id", default=None, help="Hub dataset repo (default: the dataset name)")
    ap.add_argument("--token", default=None)
    ap.add_argument("--public", action="store_true")
    ap.add_argument("--license", default=None)
    ap.add_argument("--official-link", default=None)
    ap.add_argument("--summary", default=None)
    ap.add_argument("--description", default=None)
    ap.add_argument("--remove-cache", action="store_true", help="delete --root after the push (the reference's default)")
    a = ap.parse_args(argv)
    if a.dataset not in SUPPORTED_DATASETS:
        print(f"warning: {a.dataset} is not one of {SUPPORTED_DATASETS}; check that its license allows redistribution")
    import torchvision

    cls = getattr(torchvision.datasets, a.dataset)
    dd = create_huggingface_dataset_from_torchvision(cls(a.root, train=True, download=False), cls(a.root, train=False, download=False), a.out)
    if a.push:
        full = push_to_hub(dd, a.repo_id or a.dataset, a.token, a.public, a.license, a.official_link, a.summary, a.description)
        print(f"pushed {full}")
        if a.remove_cache:
            shutil.rmtree(a.root)


if __name__ == "__main__":
    main()
