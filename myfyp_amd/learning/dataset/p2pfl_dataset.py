"""Dataset wrapper (parity: ``p2pfl/learning/dataset/p2pfl_dataset.py:55-342``).

Two backends behind one API:

* Hugging Face ``datasets`` (``Dataset``/``DatasetDict``) — the reference's representation; all
  reference constructors exist (csv/json/parquet/pandas/huggingface/generator).
* columnar numpy splits (``{"train": {"image": uint8[N,28,28], "label": int64[N]}, "test": ...}``)
  — zero-copy, used for synthetic data and for device upload: an MI355X learner uploads a whole
  partition to HBM once and never iterates rows in Python.

``generate_train_test_split`` honours ``test_size``/``seed`` (the reference ignores them,
SURVEY §2.11 #12).
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Sequence, Type, Union

import numpy as np

from myfyp_amd.learning.dataset.partition_strategies import DataPartitionStrategy

ArraySplits = Dict[str, Dict[str, np.ndarray]]
DataFilesType = Optional[Union[str, Sequence[str], Mapping[str, Union[str, Sequence[str]]]]]


class DataExportStrategy(ABC):
    """Turns one split into what a learner consumes."""

    @staticmethod
    @abstractmethod
    def export(data: Any, transforms: Optional[Callable] = None, **kwargs) -> Any: ...


def _is_hf(data: Any) -> bool:
    return type(data).__module__.startswith("datasets")


class P2PFLDataset:
    """Train/test data of one node (or of the whole federation before partitioning)."""

    def __init__(self, data: Any, train_split_name: str = "train", test_split_name: str = "test", transforms: Optional[Callable] = None) -> None:
        self._data = data
        self._train_split_name = train_split_name
        self._test_split_name = test_split_name
        self._transforms = transforms

    # ------------------------------------------------------------------ helpers
    def _is_arrays(self) -> bool:
        return isinstance(self._data, dict) and all(isinstance(v, dict) for v in self._data.values())

    def _split(self, train: bool) -> Any:
        name = self._train_split_name if train else self._test_split_name
        if self._is_arrays():
            return self._data[name]
        if _is_hf(self._data) and type(self._data).__name__ == "Dataset":
            return self._data
        return self._data[name]

    def is_split(self) -> bool:
        if self._is_arrays():
            return True
        return type(self._data).__name__ == "DatasetDict"

    def column(self, name: str, train: bool = True) -> np.ndarray:
        """Whole column of a split as a numpy array."""
        split = self._split(train)
        if isinstance(split, dict):
            return split[name]
        return np.asarray(split.with_format("numpy")[name])

    def columns(self, train: bool = True) -> List[str]:
        split = self._split(train)
        return list(split.keys()) if isinstance(split, dict) else list(split.column_names)

    # ------------------------------------------------------------------ API (reference)
    def get(self, idx: int, train: bool = True) -> Dict[str, Any]:
        split = self._split(train)
        if isinstance(split, dict):
            return {k: v[idx] for k, v in split.items()}
        return split[idx]

    def set_transforms(self, transforms: Callable) -> None:
        self._transforms = transforms

    def get_transforms(self) -> Optional[Callable]:
        return self._transforms

    def generate_train_test_split(self, test_size: float = 0.2, seed: int = 42, shuffle: bool = True, **kwargs) -> None:
        if self.is_split():
            raise ValueError("Unsupported data type (already split).")
        if isinstance(self._data, dict):
            n = len(next(iter(self._data.values())))
            idx = np.random.default_rng(seed).permutation(n) if shuffle else np.arange(n)
            n_test = int(round(n * test_size))
            test_idx, train_idx = idx[:n_test], idx[n_test:]
            self._data = {
                self._train_split_name: {k: v[train_idx] for k, v in self._data.items()},
                self._test_split_name: {k: v[test_idx] for k, v in self._data.items()},
            }
        else:
            self._data = self._data.train_test_split(test_size=test_size, seed=seed, shuffle=shuffle, **kwargs)

    def get_num_samples(self, train: bool = True) -> int:
        split = self._split(train)
        if isinstance(split, dict):
            return len(next(iter(split.values())))
        return len(split)

    def generate_partitions(self, num_partitions: int, strategy: Type[DataPartitionStrategy], seed: int = 666, label_tag: str = "label", **kwargs) -> List["P2PFLDataset"]:
        if not self.is_split():
            raise ValueError("Cannot generate partitions for single datasets. ")
        train, test = self._split(True), self._split(False)
        tr_label = {label_tag: self.column(label_tag, True)}
        te_label = {label_tag: self.column(label_tag, False)}

        class _L:  # length + label column view for strategies
            def __init__(self, d, n):
                self.d, self.n = d, n

            def __len__(self):
                return self.n

            def __getitem__(self, k):
                return self.d[k]

        tr_idx, te_idx = strategy.generate_partitions(
            _L(tr_label, self.get_num_samples(True)), _L(te_label, self.get_num_samples(False)), num_partitions, seed=seed, label_tag=label_tag, **kwargs
        )
        out = []
        for i in range(num_partitions):
            if self._is_arrays():
                a_tr = np.asarray(tr_idx[i], dtype=np.int64)
                a_te = np.asarray(te_idx[i], dtype=np.int64)
                data: Any = {
                    self._train_split_name: {k: v[a_tr] for k, v in train.items()},
                    self._test_split_name: {k: v[a_te] for k, v in test.items()},
                }
            else:
                from datasets import DatasetDict

                data = DatasetDict({self._train_split_name: train.select(tr_idx[i]), self._test_split_name: test.select(te_idx[i])})
            out.append(P2PFLDataset(data, self._train_split_name, self._test_split_name, self._transforms))
        return out

    def export(self, strategy: Type[DataExportStrategy], train: bool = True, **kwargs) -> Any:
        if not self.is_split():
            raise ValueError("Cannot export single datasets. Need to generate train/test splits first.")
        return strategy.export(self._split(train), transforms=self._transforms, **kwargs)

    # ------------------------------------------------------------------ constructors
    @classmethod
    def from_arrays(cls, train: Dict[str, np.ndarray], test: Dict[str, np.ndarray]) -> "P2PFLDataset":
        return cls({"train": dict(train), "test": dict(test)})

    @classmethod
    def from_csv(cls, data_files: DataFilesType, **kwargs) -> "P2PFLDataset":
        from datasets import load_dataset

        return cls(load_dataset("csv", data_files=data_files, **kwargs))

    @classmethod
    def from_json(cls, data_files: DataFilesType, **kwargs) -> "P2PFLDataset":
        from datasets import load_dataset

        return cls(load_dataset("json", data_files=data_files, **kwargs))

    @classmethod
    def from_parquet(cls, data_files: DataFilesType, **kwargs) -> "P2PFLDataset":
        from datasets import load_dataset

        return cls(load_dataset("parquet", data_files=data_files, **kwargs))

    @classmethod
    def from_pandas(cls, df: Any) -> "P2PFLDataset":
        from datasets import Dataset

        return cls(Dataset.from_pandas(df))

    @classmethod
    def from_huggingface(cls, dataset_name: str, **kwargs) -> "P2PFLDataset":
        from datasets import load_dataset

        return cls(load_dataset(dataset_name, **kwargs))

    @classmethod
    def from_generator(cls, generator: Callable[[], Iterable[Dict[str, Any]]]) -> "P2PFLDataset":
        from datasets import Dataset

        return cls(Dataset.from_generator(generator))
