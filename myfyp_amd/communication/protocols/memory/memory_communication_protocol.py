"""In-process transport (parity: ``protocols/memory/memory_communication_protocol.py:52-268``,
SURVEY §2.3 "In-memory protocol").

A process-global registry maps ``addr → protocol``; a send is a direct method call on the
sender's thread (like the reference). Fixes: ``stop()`` unregisters only this node (the reference
resets the whole singleton) and the registry is lock-protected. The pieces live in
the reference's module layout: ``server_singleton``, ``memory_neighbors``, ``memory_client``,
``memory_server``.
"""

from __future__ import annotations

import random

from myfyp_amd.communication.protocols.base_protocol import BaseCommunicationProtocol
from myfyp_amd.communication.protocols.client import Client
from myfyp_amd.communication.protocols.memory.memory_client import InMemoryClient
from myfyp_amd.communication.protocols.memory.memory_neighbors import InMemoryNeighbors
from myfyp_amd.communication.protocols.memory.memory_server import InMemoryServer
from myfyp_amd.communication.protocols.memory.server_singleton import ServerRegistry, ServerSingleton  # noqa: F401 (re-exports)
from myfyp_amd.communication.protocols.neighbors import Neighbors


class InMemoryCommunicationProtocol(BaseCommunicationProtocol):
    """Same API as the gRPC protocol; transport = in-process method calls."""

    def __init__(self, addr: str = "", commands=None) -> None:
        super().__init__(addr, commands)
        self._server = InMemoryServer(self)

    def parse_address(self, addr: str) -> str:
        if addr in ("", "127.0.0.1", None):
            return f"node-{random.randint(0, 10**9)}"
        return addr

    def build_neighbors(self, addr: str) -> Neighbors:
        return InMemoryNeighbors(addr)

    def build_client(self, addr: str, neighbors: Neighbors) -> Client:
        return InMemoryClient(addr, neighbors)  # type: ignore[arg-type]

    def start_transport(self) -> None:
        self._server.start()

    def stop_transport(self) -> None:
        self._server.stop()
