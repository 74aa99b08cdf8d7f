"""Framework-neutral batch export shared by the Keras/Flax export strategies: a re-iterable
sequence of ``(x, y)`` NumPy batches over one split of a P2PFLDataset."""

from __future__ import annotations

from typing import Any, Callable, Iterator, Optional, Tuple

import numpy as np


class NumpyBatches:
    def __init__(self, data: Any, train: bool, batch_size: int, shuffle: bool, seed: int = 0, transforms: Optional[Callable] = None) -> None:
        self.x = np.asarray(data.column("image", train))
        self.y = np.asarray(data.column("label", train))
        self.batch_size = max(1, int(batch_size))
        self.shuffle = shuffle
        self.transforms = transforms
        self._rng = np.random.default_rng(seed)

    def __len__(self) -> int:
        return (len(self.y) + self.batch_size - 1) // self.batch_size

    def __iter__(self) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
        order = self._rng.permutation(len(self.y)) if self.shuffle else np.arange(len(self.y))
        for i in range(0, len(order), self.batch_size):
            idx = order[i : i + self.batch_size]
            x, y = self.x[idx].astype(np.float32), self.y[idx]
            if self.transforms is not None:
                x, y = self.transforms((x, y))
            yield x, y
