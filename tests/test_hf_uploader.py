"""torchvision → Hugging Face uploader (``/root/reference/p2pfl/learning/frameworks/pytorch/utils/
torchvision_to_datasets.py``). No network and no torchvision here: the datasets are stand-ins with
torchvision's ``data`` / ``targets`` attributes, and the Hub is a recording stand-in (parity unpinned)."""

import numpy as np
import pytest

from myfyp_amd.learning.frameworks.pytorch.utils import torchvision_to_datasets as tv


class _FakeVision:
    def __init__(self, n, shape=(28, 28), seed=0):
        rng = np.random.default_rng(seed)
        self.data = rng.integers(0, 255, size=(n, *shape), dtype=np.uint8)
        self.targets = rng.integers(0, 10, size=n)

    def __len__(self):
        return len(self.targets)


def test_dataset_dict_from_torchvision_layout(tmp_path):
    import datasets

    dd = tv.create_huggingface_dataset_from_torchvision(_FakeVision(20), _FakeVision(8, seed=1), str(tmp_path / "hf"))
    assert set(dd) == {"train", "test"} and len(dd["train"]) == 20 and len(dd["test"]) == 8
    back = datasets.load_from_disk(str(tmp_path / "hf"))
    img = np.asarray(back["train"][3]["image"], dtype=np.uint8)
    assert img.shape == (28, 28) and np.array_equal(img, _FakeVision(20).data[3])
    assert back["test"][0]["label"] == int(_FakeVision(8, seed=1).targets[0])


def test_dataset_card_fields():
    card = tv.dataset_card("MNIST", license="mit", official_link="http://example.org/mnist", summary="Digits.", description="Handwritten.")
    text = str(card)
    assert "license: mit" in text and "pretty_name: MNIST" in text and "image-classification" in text
    assert "Digits." in text and "Handwritten." in text and "http://example.org/mnist" in text


def test_push_to_hub_with_stand_in_client(monkeypatch):
    import huggingface_hub

    calls = []

    class _Api:
        def login(self, token):
            calls.append(("login", token))

        def get_full_repo_name(self, repo_id, token=None):
            return f"someone/{repo_id}"

    class _DD:
        def push_to_hub(self, repo_id, private, token=None):
            calls.append(("data", repo_id, private))

    def no_load(*a, **k):
        raise OSError("offline")

    monkeypatch.setattr(huggingface_hub.DatasetCard, "load", classmethod(lambda cls, *a, **k: no_load()))
    monkeypatch.setattr(huggingface_hub.DatasetCard, "push_to_hub", lambda self, repo, repo_type=None, token=None: calls.append(("card", repo, repo_type, str(self))))
    full = tv.push_to_hub(_DD(), "MNIST", token="hf_x", public=False, license="mit", official_link="http://example.org", api=_Api())
    assert full == "someone/MNIST"
    assert calls[0] == ("login", "hf_x") and calls[1] == ("data", "MNIST", True)
    assert calls[2][:3] == ("card", "someone/MNIST", "dataset") and "license: mit" in calls[2][3]
