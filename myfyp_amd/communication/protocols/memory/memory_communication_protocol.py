"""In-process transport (parity: ``protocols/memory/*``, SURVEY §2.3 "In-memory protocol").

A process-global registry maps ``addr → protocol``; a send is a direct method call on the
sender's thread (like the reference). Fixes:

* ``stop()`` unregisters only this node (reference resets the whole singleton,
  ``memory_server.py:90-94``);
* the registry is lock-protected.
"""

from __future__ import annotations

import random
import threading
from typing import Any, Dict, List, Optional

from myfyp_amd.communication.protocols.base_protocol import BaseCommunicationProtocol
from myfyp_amd.communication.protocols.client import Client, StubClient
from myfyp_amd.communication.protocols.exceptions import NeighborNotConnectedError
from myfyp_amd.communication.protocols.neighbors import Neighbors
from myfyp_amd.management.logger import logger


class ServerRegistry:
    """Process-wide ``addr → InMemoryCommunicationProtocol`` table (reference ``ServerSingleton``)."""

    _servers: Dict[str, "InMemoryCommunicationProtocol"] = {}
    _lock = threading.Lock()

    @classmethod
    def register(cls, addr: str, proto: "InMemoryCommunicationProtocol") -> None:
        with cls._lock:
            if addr in cls._servers and cls._servers[addr] is not proto:
                raise ValueError(f"Address {addr} already in use")
            cls._servers[addr] = proto

    @classmethod
    def unregister(cls, addr: str) -> None:
        with cls._lock:
            cls._servers.pop(addr, None)

    @classmethod
    def get(cls, addr: str) -> Optional["InMemoryCommunicationProtocol"]:
        with cls._lock:
            return cls._servers.get(addr)

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            cls._servers.clear()


# Backwards-compatible name
ServerSingleton = ServerRegistry


class InMemoryNeighbors(Neighbors):
    """Direct neighbour = a reference to the peer's protocol object."""

    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> Any:
        if non_direct:
            return (None, None, self.now())
        server = ServerRegistry.get(addr)
        if server is None or not server.is_running():
            raise NeighborNotConnectedError(f"{addr} is not running")
        if handshake_msg and not server.handshake(self.self_addr):
            # already a direct neighbour there: still fine for us
            pass
        return (None, server, self.now())

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        try:
            entry = self.neis.get(addr)
            if disconnect_msg and entry is not None and entry[1] is not None:
                entry[1].remote_disconnect(self.self_addr)
        except Exception:
            pass

    def temporary_stub(self, addr: str):
        return ServerRegistry.get(addr)


class InMemoryClient(StubClient):
    """Sends by calling the peer protocol's handlers directly (generic stub client)."""


class InMemoryCommunicationProtocol(BaseCommunicationProtocol):
    """Same API as the gRPC protocol; transport = in-process method calls."""

    def parse_address(self, addr: str) -> str:
        if addr in ("", "127.0.0.1", None):
            return f"node-{random.randint(0, 10**9)}"
        return addr

    def build_neighbors(self, addr: str) -> Neighbors:
        return InMemoryNeighbors(addr)

    def build_client(self, addr: str, neighbors: Neighbors) -> Client:
        return InMemoryClient(addr, neighbors)  # type: ignore[arg-type]

    def start_transport(self) -> None:
        ServerRegistry.register(self.addr, self)
        logger.info(self.addr, f"InMemoryServer started at {self.addr}")

    def stop_transport(self) -> None:
        ServerRegistry.unregister(self.addr)
        logger.info(self.addr, f"InMemoryServer stopped at {self.addr}")

    def __init__(self, addr: str = "", commands=None) -> None:
        super().__init__(addr, commands)
