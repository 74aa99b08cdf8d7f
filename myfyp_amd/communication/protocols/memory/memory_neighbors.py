"""In-memory neighbours (parity: ``memory/memory_neighbors.py:28-109``): a direct neighbour is a
reference to the peer's protocol object, looked up in the registry."""

from __future__ import annotations

from typing import Any

from myfyp_amd.communication.protocols.exceptions import NeighborNotConnectedError
from myfyp_amd.communication.protocols.memory.server_singleton import ServerRegistry
from myfyp_amd.communication.protocols.neighbors import Neighbors


class InMemoryNeighbors(Neighbors):
    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> Any:
        if non_direct:
            return (None, None, self.now())
        server = ServerRegistry.get(addr)
        if server is None or not server.is_running():
            raise NeighborNotConnectedError(f"{addr} is not running")
        if handshake_msg:
            # False = we already are a direct neighbour there: the link is still usable
            server.handshake(self.self_addr)
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
