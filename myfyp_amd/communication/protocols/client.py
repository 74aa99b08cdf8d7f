"""Client contract (parity: ``protocols/client.py:25-89``) and the generic stub client."""

import random
import time
from abc import ABC, abstractmethod
from typing import Any, List, Optional

from myfyp_amd.management.logger import logger
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


class StubClient(Client):
    """Client over neighbour *stubs*: objects exposing ``handle_message(dict)``,
    ``handle_weights(dict)`` and ``is_running()`` — an in-process protocol, a gRPC stub wrapper or a
    cross-rank mailbox. On a transport failure the neighbour is removed (reference semantics,
    ``grpc_client.py:176-186``); a remote *command* error is reported but keeps the neighbour."""

    def __init__(self, self_addr: str, neighbors) -> None:
        super().__init__(self_addr)
        self._neighbors = neighbors

    def send(self, nei: str, msg: dict, create_connection: bool = False, raise_error: bool = False, remove_on_error: bool = True) -> None:
        from myfyp_amd.communication.protocols.exceptions import CommunicationError, NeighborNotConnectedError

        try:
            stub = None
            try:
                stub = self._neighbors.get(nei)[1]
            except KeyError:
                if not create_connection:
                    raise NeighborNotConnectedError(f"Neighbor {nei} not found.") from None
            if stub is None and create_connection:
                stub = self._neighbors.temporary_stub(nei)
            if stub is None or not stub.is_running():
                raise NeighborNotConnectedError("Neighbor not directly connected (and create_connection is false).")
            res = stub.handle_weights(msg) if "weights" in msg else stub.handle_message(msg)
            if res and "error" in res:
                raise CommunicationError(f"Error while sending a message: {msg['cmd']!r}: {res['error']!r}")
        except Exception as e:
            logger.info(self.self_addr, f"Cannot send message {msg['cmd']!r} to {nei}. Error: {e}")
            if remove_on_error and not isinstance(e, CommunicationError):
                self._neighbors.remove(nei, disconnect_msg=True)
            if raise_error:
                raise

    def broadcast(self, msg: dict, node_list: Optional[List[str]] = None) -> None:
        nodes = node_list if node_list is not None else list(self._neighbors.get_all(only_direct=True))
        for n in nodes:
            self.send(n, msg)
