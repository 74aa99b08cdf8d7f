"""Convert local image/label arrays into a Hugging Face ``DatasetDict`` (parity:
``frameworks/pytorch/utils/torchvision_to_datasets.py``, which uploads torchvision datasets to the
Hub). With no network the result is saved to disk (``save_to_disk``) — load it with
``P2PFLDataset.from_huggingface(<dir>)`` or ``datasets.load_from_disk``. ``--push`` attempts the
Hub upload (requires network + token).

    python scripts/arrays_to_hf_dataset.py --npz data.npz --out ./mnist_hf       # x_train,y_train,x_test,y_test
    python scripts/arrays_to_hf_dataset.py --synthetic mnist --out ./synthetic_mnist_hf
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", help="npz with x_train, y_train, x_test, y_test (loaded with allow_pickle=False)")
    ap.add_argument("--synthetic", choices=["mnist", "cifar10"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--push", default="", help="Hub repo id to push to (needs network)")
    a = ap.parse_args()
    import datasets
    import numpy as np

    if a.npz:
        with np.load(a.npz, allow_pickle=False) as z:
            tr, te = (z["x_train"], z["y_train"]), (z["x_test"], z["y_test"])
    else:
        from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10, synthetic_mnist

        d = synthetic_mnist() if a.synthetic == "mnist" else synthetic_cifar10()
        tr = (d.column("image", True), d.column("label", True))
        te = (d.column("image", False), d.column("label", False))
    dd = datasets.DatasetDict(
        {
            "train": datasets.Dataset.from_dict({"image": list(tr[0]), "label": tr[1].tolist()}),
            "test": datasets.Dataset.from_dict({"image": list(te[0]), "label": te[1].tolist()}),
        }
    )
    dd.save_to_disk(a.out)
    print(f"saved {dd} to {a.out}")
    if a.push:
        dd.push_to_hub(a.push)


if __name__ == "__main__":
    main()
