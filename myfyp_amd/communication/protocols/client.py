"""Client contract (parity: ``protocols/client.py:25-89``)."""

import random
import time
from abc import ABC, abstractmethod
from typing import Any, List, Optional

from myfyp_amd.settings import Settings


class Client(ABC):
    """Builds and sends messages; message dicts are transport-neutral."""

    def __init__(self, self_addr: str) -> None:
        self.self_addr = self_addr

    def build_message(self, cmd: str, args: Optional[List[str]] = None, round: Optional[int] = None) -> dict:
        """Control message. ``hash`` is unique per message (dedup key), ``ttl`` bounds relaying."""
        args = [str(a) for a in (args or [])]
        return {
            "source": self.self_addr,
            "ttl": Settings.TTL,
            "hash": hash((cmd, tuple(args), time.time_ns(), random.getrandbits(32))),
            "cmd": cmd,
            "args": args,
            "round": -1 if round is None else round,
        }

    def build_weights(self, cmd: str, round: int, serialized_model: Any, contributors: Optional[List[str]] = None, weight: int = 1) -> dict:
        """Weights message; never relayed (no ttl), like the reference protobuf ``Weights``."""
        return {
            "source": self.self_addr,
            "round": round,
            "weights": serialized_model,
            "contributors": list(contributors or []),
            "weight": weight,
            "cmd": cmd,
        }

    @abstractmethod
    def send(self, nei: str, msg: dict, create_connection: bool = False, raise_error: bool = False, remove_on_error: bool = True) -> None: ...

    @abstractmethod
    def broadcast(self, msg: dict, node_list: Optional[List[str]] = None) -> None: ...
