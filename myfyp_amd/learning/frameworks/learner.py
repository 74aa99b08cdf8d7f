"""Learner template (parity: ``p2pfl/learning/frameworks/learner.py:33-167``)."""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Dict, List, Optional, Union

import numpy as np

from myfyp_amd.learning.frameworks.callback import P2PFLCallback
from myfyp_amd.learning.frameworks.callback_factory import CallbackFactory
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel


class Learner(ABC):
    """Trains/evaluates a ``P2PFLModel`` on a ``P2PFLDataset`` for one node."""

    def __init__(self, model: P2PFLModel, data, self_addr: str = "unknown-node", aggregator=None) -> None:
        self.model: P2PFLModel = model
        self.data = data
        self._self_addr = self_addr
        self.callbacks: List[P2PFLCallback] = []
        if aggregator is not None:
            self.callbacks = CallbackFactory.create_callbacks(framework=self.get_framework(), aggregator=aggregator)
        self.epochs: int = 1

    def set_addr(self, addr: str) -> None:
        self._self_addr = addr

    def set_model(self, model: Union[P2PFLModel, List[np.ndarray], bytes]) -> None:
        if isinstance(model, P2PFLModel):
            self.model = model
        elif isinstance(model, (list, bytes, tuple)):
            self.model.set_parameters(model if not isinstance(model, tuple) else list(model))
        self.update_callbacks_with_model_info()

    def get_model(self) -> P2PFLModel:
        return self.model

    def set_data(self, data) -> None:
        self.data = data

    def get_data(self):
        return self.data

    def set_epochs(self, epochs: int) -> None:
        self.epochs = epochs

    def update_callbacks_with_model_info(self) -> None:
        info = self.model.get_info()
        for cb in self.callbacks:
            if cb.get_name() in info:
                cb.set_info(info[cb.get_name()])

    def add_callback_info_to_model(self) -> None:
        for cb in self.callbacks:
            self.model.add_info(cb.get_name(), cb.get_info())

    @abstractmethod
    def fit(self) -> P2PFLModel: ...

    @abstractmethod
    def interrupt_fit(self) -> None: ...

    @abstractmethod
    def evaluate(self) -> Dict[str, float]: ...

    @abstractmethod
    def get_framework(self) -> str: ...
