"""Collective protocol: in-process bus + cross-rank StoreBus control plane, RCCL weights plane.

Same ``CommunicationProtocol`` API as the in-memory/gRPC protocols (commands, broadcast, TTL relay,
heartbeats, neighbours), so the Node, commands and tooling are unchanged. What differs is the
workflow flavour (``workflow = "collective"``): the stages exchange weights through round-level
collectives of the process :class:`~myfyp_amd.parallel.federation.Federation` instead of gossiping
pickled models (SURVEY §2.3 "MI355X-native equivalent", §7.4 hard part 1).
"""

from __future__ import annotations

from typing import Any, Optional

from myfyp_amd.communication.protocols.memory.memory_communication_protocol import (
    InMemoryClient,
    InMemoryCommunicationProtocol,
    InMemoryNeighbors,
    ServerRegistry,
)
from myfyp_amd.communication.protocols.exceptions import NeighborNotConnectedError
from myfyp_amd.parallel.federation import Federation


class CollectiveNeighbors(InMemoryNeighbors):
    """Direct neighbour = local protocol object, or a :class:`RemotePeer` stub on another rank."""

    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> Any:
        if non_direct:
            return (None, None, self.now())
        server: Optional[Any] = ServerRegistry.get(addr)
        if server is None:
            server = Federation.get().remote_stub(addr)
        if server is None or not server.is_running():
            raise NeighborNotConnectedError(f"{addr} is not reachable")
        if handshake_msg:
            server.handshake(self.self_addr)
        return (None, server, self.now())


class CollectiveCommunicationProtocol(InMemoryCommunicationProtocol):
    """Protocol for peers whose weights move over RCCL (one process per GPU)."""

    workflow = "collective"

    def build_neighbors(self, addr: str):
        return CollectiveNeighbors(addr)

    def build_client(self, addr: str, neighbors):
        return InMemoryClient(addr, neighbors)

    def placement(self):
        """(device, mesh rank) for this peer's learner when the process drives a device mesh."""
        return Federation.get().placement()

    def bind_node(self, node) -> None:
        self.node = node
        Federation.get().register_local(node)

    def stop(self) -> None:
        inst = Federation._instance
        if inst is not None:
            node = getattr(self, "node", None)
            running = node is not None and getattr(node.state, "round", None) is not None
            inst.unregister_local(self.addr, mid_experiment=running)
        super().stop()

    def handshake(self, addr: str) -> bool:
        # remote peers connect through the StoreBus; accept both local and remote handshakes
        return self._neighbors.add(addr, non_direct=False, handshake_msg=False)
