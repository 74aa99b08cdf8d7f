"""Datasets, partitioning, wire format (reference: test/learning/p2pfl_dataset_test.py,
frameworks_test.py)."""

import pickle

import numpy as np
import pytest
import torch

from myfyp_amd.learning.dataset.p2pfl_dataset import P2PFLDataset
from myfyp_amd.learning.dataset.partition_strategies import (
    DirichletPartitionStrategy,
    LabelSkewedPartitionStrategy,
    PercentageBasedNonIIDPartitionStrategy,
    RandomIIDPartitionStrategy,
)
from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10, synthetic_mnist
from myfyp_amd.learning.frameworks.exceptions import DecodingParamsError, ModelNotMatchingError
from myfyp_amd.learning.frameworks.p2pfl_model import safe_loads
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.models import MLP, LeNet5, ResNet18


@pytest.fixture(scope="module")
def mnist():
    return synthetic_mnist(1000, 200, seed=5)


def test_synthetic_shapes(mnist):
    x = mnist.column("image", True)
    assert x.shape == (1000, 28, 28) and x.dtype == np.uint8
    assert set(np.unique(mnist.column("label", True))) <= set(range(10))
    c = synthetic_cifar10(64, 16)
    assert c.column("image", True).shape == (64, 32, 32, 3)
    assert mnist.get(3)["image"].shape == (28, 28)


@pytest.mark.parametrize("n", [1, 3, 8])
def test_iid_partitions_cover_everything(mnist, n):
    parts = mnist.generate_partitions(n, RandomIIDPartitionStrategy)
    sizes = [p.get_num_samples() for p in parts]
    assert sum(sizes) == 1000 and max(sizes) - min(sizes) <= 1
    assert sum(p.get_num_samples(train=False) for p in parts) == 200
    # same seed -> same partitions; disjoint
    again = mnist.generate_partitions(n, RandomIIDPartitionStrategy)
    assert np.array_equal(parts[0].column("label"), again[0].column("label"))


def test_dirichlet_partitions(mnist):
    parts = mnist.generate_partitions(4, DirichletPartitionStrategy, alpha=0.3, min_partition_size=10)
    assert sum(p.get_num_samples() for p in parts) == 1000
    assert min(p.get_num_samples() for p in parts) >= 10
    # huge alpha -> proportions close to the class proportions (deterministic-ish, like the reference test)
    big = mnist.generate_partitions(2, DirichletPartitionStrategy, alpha=1e10)
    assert abs(big[0].get_num_samples() - big[1].get_num_samples()) < 30
    with pytest.raises(ValueError):
        DirichletPartitionStrategy._preprocess_alpha(-1.0, 2)


def test_label_skew_and_percentage(mnist):
    parts = mnist.generate_partitions(5, LabelSkewedPartitionStrategy, shards_per_partition=2)
    assert sum(p.get_num_samples() for p in parts) == 1000
    # 2 label-sorted shards per partition: a handful of classes each (vs 10 for IID)
    assert np.mean([len(np.unique(p.column("label"))) for p in parts]) <= 4.5
    pp = mnist.generate_partitions(4, PercentageBasedNonIIDPartitionStrategy, percentage=0.3)
    for i, p in enumerate(pp):
        assert (p.column("label") == i).mean() > 0.25  # IID share would be ~0.1


def test_train_test_split_honours_args():
    d = P2PFLDataset({"image": np.zeros((100, 2, 2), np.uint8), "label": np.arange(100)})
    d.generate_train_test_split(test_size=0.3, seed=1)
    assert d.get_num_samples(True) == 70 and d.get_num_samples(False) == 30


def test_huggingface_backend_partitions():
    from datasets import Dataset, DatasetDict

    hf = DatasetDict({"train": Dataset.from_dict({"image": [[1, 2]] * 20, "label": list(range(10)) * 2}), "test": Dataset.from_dict({"image": [[0, 0]] * 4, "label": [0, 1, 2, 3]})})
    parts = P2PFLDataset(hf).generate_partitions(2, RandomIIDPartitionStrategy)
    assert [p.get_num_samples() for p in parts] == [10, 10]


def test_wire_format_roundtrip_and_errors():
    m = TorchModel(MLP(seed=1))
    blob = m.encode_parameters()
    raw = pickle.loads(blob)  # the reference format: a plain pickle dict
    assert set(raw) == {"params", "additional_info"} and len(raw["params"]) == 6
    m2 = TorchModel(MLP(seed=2))
    m2.set_parameters(blob)
    for a, b in zip(m.get_parameters(), m2.get_parameters()):
        assert np.array_equal(a, b)
    with pytest.raises(DecodingParamsError):
        m2.set_parameters(b"garbage")
    with pytest.raises(ModelNotMatchingError):
        m2.set_parameters(TorchModel(MLP(hidden_sizes=[64, 32])).get_parameters())
    copy = m.build_copy(params=blob, num_samples=5, contributors=["x"])
    assert copy.get_num_samples() == 5 and len(copy.get_parameters()) == 6


def test_safe_unpickler_refuses_code():
    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    with pytest.raises(pickle.UnpicklingError):
        safe_loads(pickle.dumps({"params": [Evil()], "additional_info": {}}))


def test_model_zoo_forward_shapes():
    x = torch.randint(0, 255, (4, 32, 32, 3), dtype=torch.uint8)
    assert LeNet5()(x).shape == (4, 10)
    assert ResNet18()(x).shape == (4, 10)
    out = MLP()(torch.randint(0, 255, (4, 28, 28), dtype=torch.uint8))
    assert torch.allclose(out.exp().sum(1), torch.ones(4), atol=1e-5)


def test_interop_adapters_and_export():
    import numpy as np

    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.flax import FlaxModel
    from myfyp_amd.learning.frameworks.learner_factory import LearnerFactory
    from myfyp_amd.learning.frameworks.simulation import try_init_learner_with_ray
    from myfyp_amd.learning.frameworks.tensorflow import KerasModel
    from myfyp_amd.learning.frameworks.torch.export import PyTorchExportStrategy
    from myfyp_amd.utils.check_ray import ray_installed

    km = KerasModel(None, params=[np.ones((2, 3), np.float32), np.zeros(3, np.float32)], num_samples=4)
    back = KerasModel(None)
    back.set_parameters(km.encode_parameters())
    assert [p.shape for p in back.get_parameters()] == [(2, 3), (3,)]
    with pytest.raises(ValueError):
        LearnerFactory.create_learner(km)
    fm = FlaxModel(None, init_params={"dense": {"kernel": np.ones((2, 2)), "bias": np.zeros(2)}})
    fm.set_parameters([np.full(2, 3.0), np.full((2, 2), 5.0)])  # sorted order: bias, kernel
    assert fm.tree["dense"]["kernel"][0, 0] == 5.0 and fm.get_framework() == "flax"
    assert ray_installed() is False
    sentinel = object()
    assert try_init_learner_with_ray(sentinel) is sentinel
    dl = PyTorchExportStrategy.export(synthetic_mnist(64, 16), batch_size=8)
    batch = next(iter(dl))
    assert batch["image"].shape == (8, 28, 28) and batch["label"].shape == (8,)
