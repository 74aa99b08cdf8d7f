"""Framework-neutral callback contract (parity: ``frameworks/callback.py:25-50``).

Aggregators declare the callbacks they need (``get_required_callbacks``); the learner instantiates
them through ``CallbackFactory``. Information flows through ``model.additional_info[name]``.
"""

from abc import ABC, abstractmethod
from typing import Any


class P2PFLCallback(ABC):
    """Named callback carrying aggregator-specific state."""

    def __init__(self) -> None:
        self.additional_info: dict = {}

    @staticmethod
    @abstractmethod
    def get_name() -> str: ...

    def set_info(self, info: Any) -> None:
        self.additional_info = dict(info) if isinstance(info, dict) else {"value": info}

    def get_info(self) -> Any:
        return self.additional_info

    # checkpoint hooks: persistent per-client state that is not part of the model
    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, state: dict) -> None:
        pass
